set -e
mkdir -p gpurun_out
for v in base t14 prio t14prio; do
  SAVQA_LIB=structured-alignment-vqa_amd/csrc/variants/libsavqa_$v.so timeout -k 10 150 python -u tools/gemm_bench.py > gpurun_out/gb_$v.log 2>&1
  echo "== $v"; cat gpurun_out/gb_$v.log
done
for v in base t14; do
  SAVQA_LIB=structured-alignment-vqa_amd/csrc/variants/libsavqa_$v.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_$v.log 2>&1
  echo "== bench $v"; tail -1 gpurun_out/bench_$v.log | cut -c1-200
done

# single-query attention (decoder cross-attention) parity + A/B against a variant library
# (usage: bash tools/gpu_q1.sh VARIANT  -> tools/ab/libsavqa_VARIANT.so)
V=${1:-prev}
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "attention" > gpurun_out/q1_tests.log 2>&1 || { tail -30 gpurun_out/q1_tests.log; exit 1; }
tail -1 gpurun_out/q1_tests.log
for r in 1 2; do
  for L in $V new; do
    if [ $L = $V ]; then export SAVQA_LIB=tools/ab/libsavqa_$V.so; else unset SAVQA_LIB; fi
    echo "== $L"
    timeout -k 10 120 python -u tools/attn_bench.py --q1 --B 256 2>&1 | grep -v amdgpu.ids
    timeout -k 10 120 python -u tools/attn_bench.py --q1 --bf16 --B 512 2>&1 | grep -v amdgpu.ids
  done
done
unset SAVQA_LIB
timeout -k 10 300 python -u bench.py --workload cfg3 --no-cpu-baseline > gpurun_out/bench_cfg3.log 2>&1 || { tail -20 gpurun_out/bench_cfg3.log; exit 1; }
tail -1 gpurun_out/bench_cfg3.log | cut -c1-200

# single-query attention (decoder cross-attention) parity + A/B against tools/ab/libsavqa_prev.so
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -k "attention" > gpurun_out/q1_tests.log 2>&1 || { tail -30 gpurun_out/q1_tests.log; exit 1; }
tail -1 gpurun_out/q1_tests.log
for r in 1 2; do
  for L in prev new; do
    if [ $L = prev ]; then export SAVQA_LIB=tools/ab/libsavqa_prev.so; else unset SAVQA_LIB; fi
    echo "== $L"
    timeout -k 10 120 python -u tools/attn_bench.py --q1 --B 256 2>&1 | grep -v amdgpu.ids
    timeout -k 10 120 python -u tools/attn_bench.py --q1 --bf16 --B 512 2>&1 | grep -v amdgpu.ids
  done
done
unset SAVQA_LIB
timeout -k 10 300 python -u bench.py --workload cfg3 --no-cpu-baseline > gpurun_out/bench_cfg3.log 2>&1 || { tail -20 gpurun_out/bench_cfg3.log; exit 1; }
tail -1 gpurun_out/bench_cfg3.log | cut -c1-200

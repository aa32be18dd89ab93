# LayerNorm forward, two rows per wave: parity, standalone timings and cfg2 / cfg3 steps vs base
set -eo pipefail
mkdir -p gpurun_out
B=tools/ab/libsavqa_base.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_blocks_gpu.py tests/test_model_gpu.py tests/test_longseq_gpu.py -k "layernorm or ln or block or golden or model or longseq" > gpurun_out/ln_tests.log 2>&1 || { tail -30 gpurun_out/ln_tests.log; exit 1; }
tail -1 gpurun_out/ln_tests.log
echo "== new"; timeout -k 10 120 python -u tools/ln_bench.py 2>&1 | grep -v amdgpu.ids
echo "== base"; SAVQA_LIB=$B timeout -k 10 120 python -u tools/ln_bench.py 2>&1 | grep -v amdgpu.ids
for r in 1 2; do
  for w in cfg2 cfg3; do
    timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('new $w', d['value'])"
    SAVQA_LIB=$B timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('base $w', d['value'])"
  done
done

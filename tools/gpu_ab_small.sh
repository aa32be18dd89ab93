# fp32 small-tile tail: GEMM parity tests, then cfg2 step A/B vs tools/ab/libsavqa_base.so
set -eo pipefail
mkdir -p gpurun_out
B=tools/ab/libsavqa_base.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k gemm > gpurun_out/gemm_tests.log 2>&1 || { tail -40 gpurun_out/gemm_tests.log; exit 1; }
tail -2 gpurun_out/gemm_tests.log
for r in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('new cfg2', d['value'])"
  SAVQA_LIB=$B timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('base cfg2', d['value'])"
done
timeout -k 10 200 python -u bench.py --workload cfg4 --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('new cfg4', d['value'])"
SAVQA_LIB=$B timeout -k 10 200 python -u bench.py --workload cfg4 --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('base cfg4', d['value'])"

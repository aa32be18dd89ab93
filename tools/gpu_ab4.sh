# lp kernel without the diagnostic branches: lp parity, per-shape A/B vs base, cfg3/cfg5 steps
set -eo pipefail
mkdir -p gpurun_out
B=tools/ab/libsavqa_base.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_lp_gpu.py > gpurun_out/lp_tests.log 2>&1 || { tail -30 gpurun_out/lp_tests.log; exit 1; }
tail -1 gpurun_out/lp_tests.log
timeout -k 10 200 python -u tools/lp_bench.py > gpurun_out/ab_lp_new.log 2>&1
SAVQA_LIB=$B timeout -k 10 200 python -u tools/lp_bench.py > gpurun_out/ab_lp_base.log 2>&1
paste -d'|' <(grep -v amdgpu gpurun_out/ab_lp_base.log | cut -c1-45) <(grep -v amdgpu gpurun_out/ab_lp_base.log | grep -o "v0 *[0-9.]*us\|savqa_lp *[0-9.]*us") <(grep -v amdgpu gpurun_out/ab_lp_new.log | grep -o "v0 *[0-9.]*us\|savqa_lp *[0-9.]*us")
for r in 1 2; do
  for w in cfg3 cfg5; do
    timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('new $w', d['value'])"
    SAVQA_LIB=$B timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('base $w', d['value'])"
  done
done

set -eo pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_lp_gpu.py -k tail 2>&1 | grep -E "passed|failed|Error|assert" | head -20
b() { timeout -k 10 300 env "$@" python -u bench.py --workload $W --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$W $*', d['value'])"; }
for W in cfg3; do for r in 1 2; do
 b SAVQA_LP_TAIL_SLABS=1
 b SAVQA_LP_TAIL_SLABS=0
done; done

set -eo pipefail
export SAVQA_BENCH_PREC=fp32x6
for p in 0 1; do echo "== pipe $p"; SAVQA_X6_PIPE=$p timeout -k 10 300 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids; done
for r in 1 2; do for p in 0 1; do
SAVQA_X6_PIPE=$p timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('pipe=$p cfg2', d['value'])"
done; done

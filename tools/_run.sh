set -eo pipefail
TO=600 bash tools/gpu.sh tests tests/test_precision_gpu.py tests/test_fullsize_gpu.py tests/test_lowp_state_gpu.py tests/test_gemm_lp_gpu.py > gpurun_out/t1.txt 2>&1 || { tail -30 gpurun_out/t1.txt; exit 1; }
tail -2 gpurun_out/t1.txt
timeout -k 10 300 python -u tools/gemm_breakdown.py cfg3 > gpurun_out/bd_base.txt 2>&1 || { tail -20 gpurun_out/bd_base.txt; exit 1; }
grep -E "total|30208x2048x512" gpurun_out/bd_base.txt
for r in 1 2; do
timeout -k 10 300 python -u bench.py --workload cfg3 --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('cfg3', d['value'])"
done

set -eo pipefail
TO=900 bash tools/gpu.sh tests tests/test_gemm_lp_gpu.py tests/test_precision_gpu.py tests/test_fullsize_gpu.py tests/test_lowp_state_gpu.py > gpurun_out/t1.txt 2>&1 || { tail -40 gpurun_out/t1.txt; exit 1; }
tail -3 gpurun_out/t1.txt
for r in 1 2; do
for w in cfg3 cfg5; do
timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());r=d['roofline'];print('$w', d['value'], r['kernel'], r['frac'])"
done
done

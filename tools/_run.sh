set -eo pipefail
TO=600 bash tools/gpu.sh tests tests/test_kernels_gpu.py -k "gather or x6 or gemm" > gpurun_out/t1.txt 2>&1 || { tail -40 gpurun_out/t1.txt; exit 1; }
tail -3 gpurun_out/t1.txt
timeout -k 10 300 python -u tools/gemm_breakdown.py cfg2 > gpurun_out/gb_cfg2.txt 2>&1
timeout -k 10 300 python -u tools/gemm_breakdown.py cfg3 > gpurun_out/gb_cfg3.txt 2>&1
for r in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());r=d['roofline'];print('cfg2', d['value'], r['kernel'], r['frac'])"
done

set -eo pipefail
TO=600 bash tools/gpu.sh tests tests/test_kernels_gpu.py -k "gemm" > gpurun_out/t_gemm.txt 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/t_gemm.txt | head; tail -30 gpurun_out/t_gemm.txt; exit 1; }
tail -2 gpurun_out/t_gemm.txt
export SAVQA_BENCH_PREC=fp32x6
for r in 1 2; do
echo "== narrow $r"; SAVQA_X6_WIDE=0 timeout -k 10 300 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids
echo "== wide $r"; SAVQA_X6_WIDE=1 timeout -k 10 300 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids
done
for r in 1 2; do
for w in 0 1; do
SAVQA_X6_WIDE=$w timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('wide=$w cfg2', d['value'])"
done
done

set -e
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k gemm 2>&1 | tail -1
bash tools/gpu_gemm_pmc.sh >/dev/null
timeout -k 10 150 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids

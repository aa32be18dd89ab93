# GEMM change check: kernel + block + model parity tests, then the per-shape step breakdown
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_blocks_gpu.py tests/test_model_gpu.py tests/test_relation_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gemm_check.log 2>&1 || { tail -40 gpurun_out/gemm_check.log; exit 1; }
tail -2 gpurun_out/gemm_check.log
timeout -k 10 300 python -u tools/gemm_breakdown.py > gpurun_out/breakdown.log 2>&1 || { tail -20 gpurun_out/breakdown.log; exit 1; }
grep -v amdgpu.ids gpurun_out/breakdown.log | head -40

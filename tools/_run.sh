set -eo pipefail
export SAVQA_BENCH_PREC=fp32x6
TO=600 bash tools/gpu.sh tests tests/test_kernels_gpu.py -k "gemm" > gpurun_out/t_gemm.txt 2>&1 || { tail -40 gpurun_out/t_gemm.txt; exit 1; }
tail -2 gpurun_out/t_gemm.txt
TO=600 bash tools/gpu.sh tests tests/test_cfg4_gpu.py > gpurun_out/t_cfg4.txt 2>&1 || { tail -60 gpurun_out/t_cfg4.txt; exit 1; }
tail -8 gpurun_out/t_cfg4.txt
TO=300 bash tools/gpu.sh ab d2 2>&1 | grep -v "amdgpu.ids\|UserWarning\|detach\|final_loss"

set -e
SAVQA_LIB=tools/ab/libsavqa_widedw.so bash tools/gpu.sh tests tests/test_kernels_gpu.py -k "gemm"
bash tools/gpu.sh ab widedw -- python -u tools/gemm_bench.py TN:1536:512:18688 TN:2048:512:18688 TN:512:2048:18688 TN:6144:512:18688 TN:1536:512:12800 TN:2048:512:12800 > gpurun_out/ab_wd.log 2>&1
grep -v "amdgpu.ids\|Warning\|final_loss\|Consider" gpurun_out/ab_wd.log | tail -40

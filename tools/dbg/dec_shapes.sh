# decoder / head GEMM shapes at cfg 3 (B = 512): bf16 lp kernel vs the fp32 kernels in use
set -e
timeout -k 10 300 python -u tools/lp_bench.py NT:512:512:512:f32 NT:512:2048:512:bf16 NT:512:512:2048:f32 NN:512:512:512:f32 NN:512:2048:512:bf16 NN:512:512:2048:f32 TN:512:512:512:atomic TN:2048:512:512:atomic TN:512:2048:512:atomic 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python -u tools/gemm_bench.py NT:512:512:512 NT:512:2048:512 NT:512:512:2048 NN:512:512:512 NN:512:2048:512 NN:512:512:2048 TN:512:512:512 TN:2048:512:512 TN:512:2048:512 2>&1 | grep -v amdgpu.ids

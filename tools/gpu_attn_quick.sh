# attention parity + timings after an attention-kernel change (usage: bash tools/gpu_attn_quick.sh)
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py tests/test_blocks_gpu.py tests/test_model_gpu.py tests/test_precision_gpu.py tests/test_attn_flash_gpu.py -k "attn or gattn or block or model or precision or golden" > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -2 gpurun_out/attn_tests.log
timeout -k 10 120 python -u tools/attn_bench.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 python -u tools/attn_bench.py --bf16 --B 512 2>&1 | grep -v amdgpu.ids

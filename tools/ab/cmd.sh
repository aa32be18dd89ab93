set -eo pipefail
timeout -k 10 300 python -u tools/lp_bench.py --variants NN:37376:2048:512:bf16 NN:37376:2048:512:bf16mask NN:37376:2048:512:bf16bits NT:37376:2048:512:bf16 2>&1 | grep -v amdgpu.ids

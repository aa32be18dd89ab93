set -eo pipefail
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_fullsize_gpu.py tests/test_cfg4_gpu.py tests/test_ddp_gpu.py tests/test_relation_gpu.py 2>&1 | grep -E "wide-range|passed|failed|Error|assert" | head -40

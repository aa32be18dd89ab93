# data-path rows: device collate + GQA reader + train loop tests (usage: bash tools/gpu_data.sh)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_collate_gpu.py tests/test_train_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/data_tests.log 2>&1 || { tail -60 gpurun_out/data_tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/data_tests.log | tail -15

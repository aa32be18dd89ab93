set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_collate_gpu.py tests/test_train_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/collate_tests.log 2>&1 || { tail -60 gpurun_out/collate_tests.log; exit 1; }
tail -15 gpurun_out/collate_tests.log
timeout -k 10 300 python -u tools/collate_bench.py > gpurun_out/collate_bench.log 2>&1 || { tail -30 gpurun_out/collate_bench.log; exit 1; }
cat gpurun_out/collate_bench.log

# collate row: GPU parity tests, bench, kernel-trace profile (usage: bash tools/gpu_collate.sh)
set -e
mkdir -p gpurun_out/collate_prof
timeout -k 10 300 python -u -m pytest tests/test_collate_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/collate_tests.log 2>&1 || { tail -60 gpurun_out/collate_tests.log; exit 1; }
tail -3 gpurun_out/collate_tests.log
timeout -k 10 300 python -u tools/collate_bench.py > gpurun_out/collate_bench.log 2>&1 || { tail -30 gpurun_out/collate_bench.log; exit 1; }
cat gpurun_out/collate_bench.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/collate_prof -o run -- python3 -u tools/collate_bench.py > gpurun_out/collate_prof.log 2>&1 || { tail -30 gpurun_out/collate_prof.log; exit 1; }
grep -i "collate\|Name" gpurun_out/collate_prof/run_kernel_stats.csv | cut -c1-200

set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_lp_gpu.py 2>&1 | tee gpurun_out/lp_tests.log | tail -15
timeout -k 10 200 python -u tools/lp_bench.py --variants 2>&1 | tee gpurun_out/lp_bench_variants.txt

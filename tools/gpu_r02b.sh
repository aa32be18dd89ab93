# lp GEMM tests + variant bench (incl. masked / residual epilogues) + cfg3 breakdown + graph
# capture test (usage: bash tools/gpu_r02b.sh)
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_lp_gpu.py 2>&1 | tee gpurun_out/lp_tests.log | tail -3
timeout -k 10 200 python -u tools/lp_bench.py --variants 2>&1 | tee gpurun_out/lp_bench_variants.txt
timeout -k 10 200 python -u tools/gemm_breakdown.py cfg3 > gpurun_out/breakdown_cfg3.txt 2>&1
head -16 gpurun_out/breakdown_cfg3.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_graph_capture_gpu.py 2>&1 | tee gpurun_out/graph_test.log | tail -30

# new parity tests (cfg2 vs oracle, super-node relation golden, DDP equivalence) + per-shape
# GEMM breakdowns of cfg3 / cfg5 (usage: bash tools/gpu_r02a.sh)
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_ddp_gpu.py::test_two_ranks_on_half_batches_equal_one_rank_on_the_batch tests/test_graph_capture_gpu.py 2>&1 | tee gpurun_out/newtests.log || { tail -40 gpurun_out/newtests.log; exit 1; }
grep -E "passed|cfg2 B=256" gpurun_out/newtests.log
for w in cfg3 cfg5; do
  timeout -k 10 200 python -u tools/gemm_breakdown.py $w > gpurun_out/breakdown_$w.txt 2>&1 || { tail -20 gpurun_out/breakdown_$w.txt; exit 1; }
  head -25 gpurun_out/breakdown_$w.txt
done
timeout -k 10 200 python -u tools/lp_bench.py --variants > gpurun_out/lp_bench_variants.txt 2>&1 || { tail -20 gpurun_out/lp_bench_variants.txt; exit 1; }
cat gpurun_out/lp_bench_variants.txt

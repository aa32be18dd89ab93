set -e
for sp in -1 1 2 3 4 6 8 12 16; do
  echo "== split $sp"
  SAVQA_BENCH_SPLIT=$sp timeout -k 10 100 python -u tools/gemm_bench.py TN:6144:512:18688 TN:512:2048:18688 TN:1536:512:18688 2>&1 | grep -v amdgpu.ids
done

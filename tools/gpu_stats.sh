# kernel-trace stats of bench workloads (usage: bash tools/gpu_stats.sh cfg2 cfg3 ...)
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for w in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats_$w -o run -- python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/stats_$w.log 2>&1
  echo "$w done"
done

# bench lines of the cfg4 and super-node relation workloads (usage: bash tools/gpu_other_lines.sh)
set -eo pipefail
mkdir -p gpurun_out
for w in cfg4 rel; do
  timeout -k 10 400 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/bench_$w.log 2>&1 || { tail -20 gpurun_out/bench_$w.log; exit 1; }
  tail -1 gpurun_out/bench_$w.log | cut -c1-160
done

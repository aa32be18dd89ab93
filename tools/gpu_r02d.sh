# full GPU suite + smoke + bench lines of every workload + rocprof profiles of cfg2/cfg3/cfg5
set -e
mkdir -p gpurun_out
bash tools/gpu_round.sh
bash tools/gpu_workloads.sh
for w in cfg2 cfg3 cfg5; do bash tools/profile_round.sh r02 $w; done

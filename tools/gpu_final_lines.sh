# Round-end check: full GPU suite + smoke, then the bench line of every workload (cfg2 with the
# CPU baseline: the driver's default command)
set -eo pipefail
mkdir -p gpurun_out
bash tools/gpu_suite.sh
timeout -k 10 400 python -u bench.py > gpurun_out/bench_cfg2.json 2> gpurun_out/bench_cfg2.err || { tail -20 gpurun_out/bench_cfg2.err; exit 1; }
tail -c 600 gpurun_out/bench_cfg2.json
WORKLOADS="cfg3 cfg5 cfg4 rel" bash tools/gpu_workloads.sh

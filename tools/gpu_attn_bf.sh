# bf16 MFMA attention: parity + kernel timings + cfg3/cfg5 bench lines (usage: bash tools/gpu_attn_bf.sh)
set -eo pipefail
mkdir -p gpurun_out
bash tools/gpu_attn_quick.sh
timeout -k 10 300 python -u bench.py --workload cfg3 --no-cpu-baseline > gpurun_out/bench_cfg3.log 2>&1 || { tail -20 gpurun_out/bench_cfg3.log; exit 1; }
tail -1 gpurun_out/bench_cfg3.log
timeout -k 10 300 python -u bench.py --workload cfg5 --no-cpu-baseline > gpurun_out/bench_cfg5.log 2>&1 || { tail -20 gpurun_out/bench_cfg5.log; exit 1; }
tail -1 gpurun_out/bench_cfg5.log

# Session re-entry check: full GPU suite + smoke, per-shape lp GEMM rates, cfg2/cfg3 bench lines
set -eo pipefail
mkdir -p gpurun_out
bash tools/gpu_suite.sh
timeout -k 10 300 python -u tools/lp_bench.py > gpurun_out/lp_bench.log 2>&1 || { tail -20 gpurun_out/lp_bench.log; exit 1; }
for w in cfg2 cfg3; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err
  python -c "import json;d=json.load(open('gpurun_out/bench_$w.json'));print('$w', d['value'],d['ms_per_step'],(d.get('roofline') or {}).get('frac'))"
done

# bench lines of the other workloads (cfg 3 bf16, cfg 5 fp8+bf16, cfg 4 stress shape, relation branch)
set -e
mkdir -p gpurun_out
for w in ${WORKLOADS:-cfg3 cfg5 cfg4 rel}; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err
  echo "$w: $(python -c "import json;d=json.load(open('gpurun_out/bench_$w.json'));print(d['value'],d['ms_per_step'],d['dtype'],(d.get('roofline') or {}).get('frac'))")"
done

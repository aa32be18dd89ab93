set -eo pipefail
timeout -k 10 400 python -u bench.py > gpurun_out/bench_cfg2.json 2> gpurun_out/bench_cfg2.err
for w in cfg3 cfg4 cfg5 rel; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err
done
for w in cfg2 cfg3 cfg4 cfg5 rel; do python -c "import json;d=json.load(open('gpurun_out/bench_$w.json'));r=d['roofline'];print('$w', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('traffic'), (d.get('cpu_baseline') or {}).get('value'))"; done

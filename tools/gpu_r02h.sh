set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_attn_flash_gpu.py tests/test_blocks_gpu.py tests/test_kernels_gpu.py tests/test_longseq_gpu.py tests/test_relation_gpu.py 2>&1 | tee gpurun_out/attn_tests.log | tail -3
for w in cfg2 cfg3 cfg4 rel; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err
  python -c "import json;d=json.load(open('gpurun_out/bench_$w.json'));print('$w', d['value'],d['ms_per_step'],(d.get('roofline') or {}).get('frac'))"
done

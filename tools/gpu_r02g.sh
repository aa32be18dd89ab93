set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_blocks_gpu.py tests/test_fullsize_gpu.py 2>&1 | tee gpurun_out/k_tests.log | tail -4
for w in cfg2 cfg3; do
  timeout -k 10 200 python -u tools/gemm_breakdown.py $w > gpurun_out/breakdown_$w.txt 2>&1
  grep -E "total|skinny" gpurun_out/breakdown_$w.txt | head -12
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_cfg2.json 2> gpurun_out/bench_cfg2.err
python -c "import json;d=json.load(open('gpurun_out/bench_cfg2.json'));print('cfg2', d['value'],d['ms_per_step'],(d.get('roofline') or {}).get('frac'))"
timeout -k 10 300 python -u bench.py --workload cfg3 --no-cpu-baseline > gpurun_out/bench_cfg3.json 2> gpurun_out/bench_cfg3.err
python -c "import json;d=json.load(open('gpurun_out/bench_cfg3.json'));print('cfg3', d['value'],d['ms_per_step'],(d.get('roofline') or {}).get('frac'))"

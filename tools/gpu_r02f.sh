set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_lp_gpu.py tests/test_precision_gpu.py tests/test_graph_capture_gpu.py tests/test_kernels_gpu.py 2>&1 | tee gpurun_out/lp_tests.log | tail -15
for w in cfg3 cfg5; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err
  python -c "import json;d=json.load(open('gpurun_out/bench_$w.json'));print('$w', d['value'],d['ms_per_step'],(d.get('roofline') or {}).get('frac'), (d.get('roofline') or {}).get('kernel'))"
done
timeout -k 10 200 python -u tools/gemm_breakdown.py cfg3 > gpurun_out/breakdown_cfg3.txt 2>&1
head -14 gpurun_out/breakdown_cfg3.txt

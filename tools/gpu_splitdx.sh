# split-K scatter-add dX (GloVe-table gradient): parity tests + in-step GEMM breakdown + bench
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_train_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/splitdx_tests.log 2>&1 || { tail -30 gpurun_out/splitdx_tests.log; exit 1; }
tail -1 gpurun_out/splitdx_tests.log
timeout -k 10 200 python -u tools/gemm_breakdown.py > gpurun_out/gb_splitdx.txt 2>&1
grep -E "total|3584x300|46080x300|15104x" gpurun_out/gb_splitdx.txt
timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-roofline > gpurun_out/bench_splitdx.json 2> gpurun_out/bench_splitdx.err
python -c "import json;d=json.load(open('gpurun_out/bench_splitdx.json'));print(d['value'],d['ms_per_step'])"

set -eo pipefail
TO=900 bash tools/gpu.sh tests tests/test_gemm_lp_gpu.py tests/test_cfg4_gpu.py > gpurun_out/t1.txt 2>&1 || { tail -40 gpurun_out/t1.txt; exit 1; }
tail -12 gpurun_out/t1.txt
for r in 1 2; do
for s in 0 1; do
SAVQA_LP_SLABS=$s timeout -k 10 300 python -u bench.py --workload cfg3 --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('slabs=$s cfg3', d['value'])"
done
SAVQA_LIB=tools/ab/libsavqa_d2.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('d2 cfg2', d['value'])"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('d1 cfg2', d['value'])"
done
timeout -k 10 400 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
python -c "import json;d=json.load(open('gpurun_out/bench_full.json'));print(d['value'], json.dumps(d['roofline'])[:3000]); print(d['cpu_baseline'])"

set -eo pipefail
TO=600 bash tools/gpu.sh tests tests/test_lowp_state_gpu.py tests/test_precision_gpu.py tests/test_model_gpu.py tests/test_train_gpu.py > gpurun_out/t1.txt 2>&1 || { tail -40 gpurun_out/t1.txt; exit 1; }
tail -3 gpurun_out/t1.txt
for r in 1 2; do
for v in 1 0; do
SAVQA_ADAM_SHADOW=$v timeout -k 10 300 python -u bench.py --workload cfg3 --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('shadow=$v cfg3', d['value'])"
done; done

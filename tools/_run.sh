set -eo pipefail
TO=600 bash tools/gpu.sh tests tests/test_relation_gpu.py tests/test_kernels_gpu.py -k "rel or relation" > gpurun_out/t1.txt 2>&1 || { tail -30 gpurun_out/t1.txt; exit 1; }
tail -2 gpurun_out/t1.txt
for r in 1 2; do for L in tools/ab/libsavqa_relold.so structured-alignment-vqa_amd/libsavqa.so; do
SAVQA_LIB=$L timeout -k 10 300 python -u bench.py --workload rel --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$L rel', d['value'])"
done; done

set -eo pipefail
TO=600 bash tools/gpu.sh tests tests/test_kernels_gpu.py tests/test_precision_gpu.py -k "attention or bf16 or precision" > gpurun_out/t1.txt 2>&1 || { tail -40 gpurun_out/t1.txt; exit 1; }
tail -2 gpurun_out/t1.txt
for r in 1 2; do
for L in structured-alignment-vqa_amd/libsavqa.so tools/ab/libsavqa_bf2w4.so; do
echo "== $L"; SAVQA_LIB=$L timeout -k 10 200 python -u tools/attn_bench.py --bf16 --B 512 2>&1 | grep -v amdgpu.ids
done
done
for r in 1 2; do
for L in structured-alignment-vqa_amd/libsavqa.so tools/ab/libsavqa_bf2w4.so; do
SAVQA_LIB=$L timeout -k 10 300 python -u bench.py --workload cfg3 --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$L cfg3', d['value'])"
done
done

set -eo pipefail
TO=400 bash tools/gpu.sh tests tests/test_kernels_gpu.py -k "attention or attn" > gpurun_out/t1.txt 2>&1 || { tail -30 gpurun_out/t1.txt; exit 1; }
tail -2 gpurun_out/t1.txt
for r in 1 2; do
for v in base attnold; do
L=structured-alignment-vqa_amd/libsavqa.so; [ $v != base ] && L=tools/ab/libsavqa_$v.so
echo "== $v"; SAVQA_LIB=$L timeout -k 10 120 python -u tools/attn_bench.py --bf16 --B 512 --T 73 50 2>&1 | grep -v amdgpu.ids
SAVQA_LIB=$L timeout -k 10 120 python -u tools/attn_bench.py --B 256 --T 73 50 2>&1 | grep -v amdgpu.ids
done; done
for r in 1 2; do
for v in base attnold; do
L=structured-alignment-vqa_amd/libsavqa.so; [ $v != base ] && L=tools/ab/libsavqa_$v.so
for w in cfg2 cfg3; do
SAVQA_LIB=$L timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$v $w', d['value'])"
done; done; done

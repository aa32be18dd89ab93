set -eo pipefail
TO=600 bash tools/gpu.sh tests tests/test_kernels_gpu.py -k "attention or q1" > gpurun_out/t1.txt 2>&1 || { tail -40 gpurun_out/t1.txt; exit 1; }
tail -2 gpurun_out/t1.txt
for r in 1 2; do
for L in tools/ab/libsavqa_attnold.so structured-alignment-vqa_amd/libsavqa.so; do
echo "== $L"
SAVQA_LIB=$L timeout -k 10 200 python -u tools/attn_bench.py --q1 --B 256 --T 73 50 2>&1 | grep -v amdgpu.ids
SAVQA_LIB=$L timeout -k 10 200 python -u tools/attn_bench.py --q1 --bf16 --B 512 --T 73 50 2>&1 | grep -v amdgpu.ids
done
done

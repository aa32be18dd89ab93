set -eo pipefail
TO=600 bash tools/gpu.sh tests tests/test_kernels_gpu.py tests/test_attn_flash_gpu.py tests/test_model_gpu.py tests/test_blocks_gpu.py tests/test_precision_gpu.py tests/test_longseq_gpu.py > gpurun_out/t1.txt 2>&1 || { tail -40 gpurun_out/t1.txt; exit 1; }
tail -3 gpurun_out/t1.txt
for r in 1 2; do
echo "== old"; SAVQA_LIB=tools/ab/libsavqa_attnold.so timeout -k 10 200 python -u tools/attn_bench.py --bf16 --B 512 2>&1 | grep -v amdgpu.ids
SAVQA_LIB=tools/ab/libsavqa_attnold.so timeout -k 10 200 python -u tools/attn_bench.py --B 256 2>&1 | grep -v amdgpu.ids
echo "== new"; timeout -k 10 200 python -u tools/attn_bench.py --bf16 --B 512 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python -u tools/attn_bench.py --B 256 2>&1 | grep -v amdgpu.ids
done
for r in 1 2; do
SAVQA_LIB=tools/ab/libsavqa_attnold.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('old cfg2', d['value'])"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('new cfg2', d['value'])"
done

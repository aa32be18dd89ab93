set -eo pipefail
SAVQA_X6_PERSIST=1 TO=600 bash tools/gpu.sh tests tests/test_kernels_gpu.py -k "gemm" > gpurun_out/t1.txt 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/tests.log | head -10; tail -5 gpurun_out/t1.txt; exit 1; }
tail -1 gpurun_out/t1.txt
export SAVQA_BENCH_PREC=fp32x6
S="NT:18688:2048:512 NN:18688:2048:512 NT:18688:1536:512 NT:18688:512:2048 TN:2048:512:18688 NT:18688:6144:512"
for r in 1 2; do
echo "== base"; SAVQA_LIB=tools/ab/libsavqa_relold.so timeout -k 10 200 python -u tools/gemm_bench.py $S 2>&1 | grep -v amdgpu.ids | cut -c1-70
for p in 0 1; do echo "== new persist $p"; SAVQA_X6_PERSIST=$p timeout -k 10 200 python -u tools/gemm_bench.py $S 2>&1 | grep -v amdgpu.ids | cut -c1-70; done
done
for r in 1 2; do
SAVQA_LIB=tools/ab/libsavqa_relold.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('base cfg2', d['value'])"
for p in 0 1; do SAVQA_X6_PERSIST=$p timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('persist=$p cfg2', d['value'])"; done
done

set -eo pipefail
S="NT:512:512:512 NT:512:2048:512 NT:512:512:2048 NN:512:512:512 NN:512:2048:512 NN:512:512:2048 TN:512:512:512 TN:2048:512:512 TN:512:2048:512 NT:1024:512:512 NT:1024:2048:512 NN:1024:512:2048"
echo "== fp32 skinny (x6 mode)"; SAVQA_BENCH_PREC=fp32x6 timeout -k 10 200 python -u tools/gemm_bench.py $S 2>&1 | grep -v amdgpu.ids
echo "== bf16x3 + torch bf16 yardstick"; SAVQA_BENCH_PREC=bf16x3 timeout -k 10 200 python -u tools/gemm_bench.py $S 2>&1 | grep -v amdgpu.ids

set -e
S="NT:18688:2048:512 NT:18688:1536:512 NT:18688:6144:512 NN:18688:512:2048 NN:18688:2048:512 NN:18688:512:6144 TN:2048:512:18688 TN:6144:512:18688 TN:1536:512:18688 NT:12800:2048:512 NT:12800:512:2048 NT:4096:4096:4096"
echo "== sk" >> gpurun_out/var4.log
timeout -k 10 120 python tools/gemm_bench.py $S >> gpurun_out/var4.log 2>&1
echo "== dp" >> gpurun_out/var4.log
SAVQA_GEMM_SK=0 timeout -k 10 120 python tools/gemm_bench.py $S >> gpurun_out/var4.log 2>&1

set -e
S="NT:18688:2048:512 NT:18688:1536:512 NT:18688:6144:512 NN:18688:512:2048 NN:18688:2048:512 NN:18688:512:6144 TN:2048:512:18688 TN:6144:512:18688 NT:12800:2048:512 NT:4096:4096:4096"
for v in pf2 pf2bk32 mi32; do
  echo "== $v" >> gpurun_out/var7.log
  SAVQA_LIB=structured-alignment-vqa_amd/csrc/build/libsavqa_$v.so timeout -k 10 120 python tools/gemm_bench.py $S >> gpurun_out/var7.log 2>&1
done

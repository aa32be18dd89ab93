set -e
SAVQA_LIB=structured-alignment-vqa_amd/csrc/variants/libsavqa_dw64k32.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k gemm 2>&1 | tail -1
SAVQA_LIB=structured-alignment-vqa_amd/csrc/variants/libsavqa_dw64k16.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k gemm 2>&1 | tail -1
for rep in 1 2; do
for v in dw128 dw64k32 dw64k16; do
  echo "== $v $rep"
  SAVQA_LIB=structured-alignment-vqa_amd/csrc/variants/libsavqa_$v.so timeout -k 10 150 python -u tools/gemm_bench.py TN:1536:512:18688 TN:2048:512:18688 TN:512:2048:18688 TN:6144:512:18688 TN:1536:512:12800 TN:6144:512:12800 2>&1 | grep -v amdgpu.ids | awk '{print $1, $8, $9}'
done
done

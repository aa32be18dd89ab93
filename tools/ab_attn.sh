# attention A/B (usage: bash tools/ab_attn.sh NAME...): parity tests on the first, then timings
set -e
SAVQA_LIB=structured-alignment-vqa_amd/csrc/variants/libsavqa_$1.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_blocks_gpu.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -1
for rep in 1 2; do for v in "$@"; do
  echo "== $v $rep"; SAVQA_LIB=structured-alignment-vqa_amd/csrc/variants/libsavqa_$v.so timeout -k 10 120 python -u tools/attn_bench.py 2>&1 | grep -v amdgpu.ids
done; done

# interleaved A/B, 3 rounds (usage: bash tools/ab_gemm2.sh NAME...)
set -e
for rep in 1 2 3; do
for v in "$@"; do
  lib=structured-alignment-vqa_amd/csrc/variants/libsavqa_$v.so
  echo "== $v $rep $(SAVQA_LIB=$lib timeout -k 10 150 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids | awk '{s+=$8} END {print s " us total"}')"
done
done

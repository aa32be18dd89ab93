# A/B of GEMM variants built by tools/build_variants.sh (usage: bash tools/ab_gemm.sh NAME...)
set -e
mkdir -p gpurun_out
for v in "$@"; do
  lib=structured-alignment-vqa_amd/csrc/variants/libsavqa_$v.so
  [ "$v" = cur ] && lib=structured-alignment-vqa_amd/libsavqa.so
  SAVQA_LIB=$lib timeout -k 10 150 python -u tools/gemm_bench.py > gpurun_out/gb_$v.log 2>&1
  echo "== $v"; grep -v amdgpu.ids gpurun_out/gb_$v.log
done

# A/B of library variants on the real step's GEMMs (usage: bash tools/ab_breakdown.sh NAME...)
set -e
mkdir -p gpurun_out
for rep in 1 2; do
for v in "$@"; do
  lib=structured-alignment-vqa_amd/csrc/variants/libsavqa_$v.so
  [ "$v" = cur ] && lib=structured-alignment-vqa_amd/libsavqa.so
  SAVQA_LIB=$lib timeout -k 10 200 python -u tools/gemm_breakdown.py > gpurun_out/bd_$v.log 2>&1
  echo "== $v rep $rep: $(grep total gpurun_out/bd_$v.log)"
  grep -E "NN 18688x2048x512 m|NT 18688x512x2048 br|NT 18688x2048x512 bR" gpurun_out/bd_$v.log | awk '{print "   ", $1, $5, $6, $10, $11, $12}'
done
done

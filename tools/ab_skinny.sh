# skinny-GEMM A/B (usage: bash tools/ab_skinny.sh NAME...; cur = in-tree library)
set -e
mkdir -p gpurun_out
S="NN:256:512:2048 NN:256:512:512 TN:512:512:256 NT:256:512:2048 NT:256:2048:512 TN:2048:512:256 NN:256:2048:512 NT:256:512:512 TN:512:2048:256"
for v in "$@"; do
  lib=structured-alignment-vqa_amd/csrc/variants/libsavqa_$v.so
  [ "$v" = cur ] && lib=structured-alignment-vqa_amd/libsavqa.so
  echo "== $v"
  SAVQA_LIB=$lib timeout -k 10 150 python -u tools/gemm_bench.py $S 2>&1 | grep -v amdgpu.ids | awk '{print $1, $6, $7}'
done

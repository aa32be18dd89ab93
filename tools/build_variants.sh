#!/bin/bash
# Build alternative libsavqa.so variants (same ABI) for A/B timing via SAVQA_LIB=...
# usage: tools/build_variants.sh NAME "-DFLAG=.. ..." [NAME "FLAGS"]...
# objects under csrc/build (gpurun-ignored); the .so goes to csrc/variants/ (travels, git-ignored)
set -e
cd "$(dirname "$0")/../structured-alignment-vqa_amd/csrc"
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  out=build/var_$name; mkdir -p $out
  for f in capi.cpp gemm.hip gemm_bf16.hip ln.hip attn.hip attn_flash.hip misc.hip dropout.hip rel.hip collate.hip; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $flags -c $f -o $out/$f.o &
  done
  wait
  mkdir -p variants
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $out/*.o -o variants/libsavqa_$name.so
  echo built csrc/variants/libsavqa_$name.so
done

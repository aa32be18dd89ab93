# Build a variant libsavqa with attn.hip compiled under extra -D flags (A/B via SAVQA_LIB).
# usage: bash tools/build_attn_variant.sh NAME "-DFOO=1 -DBAR=2"   (run from the repo root, CPU)
set -e
NAME=$1; DEFS=$2
C=structured-alignment-vqa_amd/csrc
O=/tmp/abobj/$NAME; mkdir -p $O tools/ab
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $DEFS -c $C/attn.hip -o $O/attn.hip.o
OBJS=$(ls $C/build/*.o | grep -v '/attn.hip.o')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS $O/attn.hip.o -o tools/ab/libsavqa_$NAME.so
echo built tools/ab/libsavqa_$NAME.so

# Build a variant libsavqa with some source files compiled under extra -D flags, for interleaved
# A/B runs through SAVQA_LIB (tools/gpu.sh ab). Run from the repo root on the CPU, after `make`.
# usage: bash tools/build_variant.sh NAME "SOURCE.hip [SOURCE.hip ...]" "-DFOO=1 -DBAR=2"
set -e
NAME=$1; SRCS=$2; DEFS=$3
C=structured-alignment-vqa_amd/csrc
O=/tmp/abobj/$NAME; rm -rf $O; mkdir -p $O tools/ab
OBJS=$(ls $C/build/*.o)
for SRC in $SRCS; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $DEFS -c $C/$SRC -o $O/$SRC.o
  OBJS=$(echo "$OBJS" | grep -v "/$SRC.o")
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS $O/*.o -o tools/ab/libsavqa_$NAME.so
echo built tools/ab/libsavqa_$NAME.so

# Build a variant libsavqa with ONE source file compiled under extra -D flags, for interleaved
# A/B runs through SAVQA_LIB (tools/gpu.sh ab). Run from the repo root on the CPU, after `make`.
# usage: bash tools/build_variant.sh NAME SOURCE.hip "-DFOO=1 -DBAR=2"
set -e
NAME=$1; SRC=$2; DEFS=$3
C=structured-alignment-vqa_amd/csrc
O=/tmp/abobj/$NAME; mkdir -p $O tools/ab
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $DEFS -c $C/$SRC -o $O/$SRC.o
OBJS=$(ls $C/build/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS $O/$SRC.o -o tools/ab/libsavqa_$NAME.so
echo built tools/ab/libsavqa_$NAME.so

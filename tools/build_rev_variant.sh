#!/bin/bash
# tools/build_rev_variant.sh REV NAME [FLAGS] -- abl/NAME/libgtsmax_hip.so with
# smax_kernels.hip as of git revision REV (the other objects from the in-tree
# build): the A side of an interleaved A/B against the working tree
# (tools/gpu_round.sh abm:...).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
M=$R/genometools_smax_amd
REV=$1; NAME=$2; FLAGS=${3:-}
make -s -C "$M" >/dev/null
mkdir -p "$R/abl/$NAME" "$M/build/var"
SRC=$M/build/var/$NAME.hip
git -C "$R" show "$REV:genometools_smax_amd/csrc/smax_kernels.hip" > "$SRC"
OBJS="$M/build/smax_runtime.o $M/build/esa_build.o $M/build/esa_build64.o $M/build/esa_write.o $M/build/maxpairs.o $M/build/repfind_lines.o $M/build/lcpitv.o $M/build/synth.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I"$R/include" -I"$M/host" -I"$M/csrc" \
  -DGT_SMAX_BUILD_ID="\"rev-$NAME\"" $FLAGS -c -o "$M/build/var/$NAME.o" "$SRC"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o "$R/abl/$NAME/libgtsmax_hip.so" \
  "$M/build/var/$NAME.o" $OBJS -lpthread -ldl
echo "built abl/$NAME (smax_kernels.hip at $REV)"

#!/bin/bash
# Build A/B variants of the library that differ only in smax_kernels.hip's
# K1 build switches: tools/build_variants.sh NAME "-DSMAX_X=1 ..." [NAME FLAGS ...]
# -> abl/NAME/libgtsmax_hip.so (the other objects from the in-tree build)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
M=$R/genometools_smax_amd
make -s -C "$M" >/dev/null
OBJS="$M/build/smax_runtime.o $M/build/esa_build.o $M/build/esa_build64.o $M/build/esa_write.o $M/build/maxpairs.o $M/build/repfind_lines.o $M/build/lcpitv.o $M/build/synth.o"
pids=()
while [ $# -ge 2 ]; do
  NAME=$1; FLAGS=$2; shift 2
  mkdir -p "$R/abl/$NAME" "$M/build/var"
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -I"$R/include" -I"$M/host" \
      -DGT_SMAX_BUILD_ID="\"var-$NAME\"" -mllvm -amdgpu-atomic-optimizer-strategy=None $FLAGS -c -o "$M/build/var/$NAME.o" "$M/csrc/smax_kernels.hip" &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o "$R/abl/$NAME/libgtsmax_hip.so" \
      "$M/build/var/$NAME.o" $OBJS -lpthread -ldl && echo "built abl/$NAME ($FLAGS)" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done

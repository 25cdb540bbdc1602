#!/bin/sh
# build.sh -- links the reference-side binding into an executable test:
# integration/esa_linsmax.c compiled against the reference's headers (as
# check_shim.sh does) + gt_stubs.c (test doubles of the reader, GtError and
# allocator) + shim_driver.c, linked with libgtsmax_hip.so.  Output:
# integration/exec_test/_build/shim_exec (git-ignored; it travels to the GPU
# box with the tree, where tests/test_shim_exec_gpu.py runs it).  Needs the
# reference tree for its headers only; nothing of it is built or linked.
set -eu
REF=${1:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
INTEG=$(dirname "$HERE")
ROOT=$(dirname "$INTEG")
OUT=$HERE/_build
T=$(mktemp -d)
trap 'rm -rf "$T"' EXIT
mkdir -p "$T/src/match" "$OUT"
cp "$INTEG/esa_linsmax.c" "$INTEG/esa_linsmax.h" "$T/src/match/"
CFLAGS="-std=c99 -O2 -Wall -Wextra -Wno-unused-parameter -Werror -D_GNU_SOURCE"
INC="-I$T/src -I$REF/src -I$ROOT/include"
gcc $CFLAGS $INC -c -o "$T/esa_linsmax.o" "$T/src/match/esa_linsmax.c"
gcc $CFLAGS $INC -c -o "$T/gt_stubs.o" "$HERE/gt_stubs.c"
gcc $CFLAGS $INC -c -o "$T/shim_driver.o" "$HERE/shim_driver.c"
gcc -o "$OUT/shim_exec" "$T/shim_driver.o" "$T/esa_linsmax.o" "$T/gt_stubs.o" \
    -L"$ROOT/genometools_smax_amd/lib" -lgtsmax_hip \
    -Wl,-rpath,'$ORIGIN/../../../genometools_smax_amd/lib'
echo "built $OUT/shim_exec"

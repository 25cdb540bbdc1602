#!/bin/sh
# check_shim.sh -- compile the reference-side binding against the reference.
#
# Stages integration/esa_linsmax.{c,h} as src/match/ and the reference's
# src/tools/gt_repfind.c with integration/gt_repfind_smax.patch applied in an
# overlay directory, and compiles both to object files with gcc against the
# reference's own headers (first the overlay, then $REF/src) plus this repo's
# include/ -- the way the reference's build compiles its sources (C99, 64-bit
# GtUword).  Nothing of the reference is built or linked; its tree is only
# read.  Exit status 0 = both translation units compile without warnings.
set -eu
REF=${1:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(dirname "$HERE")
T=$(mktemp -d)
trap 'rm -rf "$T"' EXIT
mkdir -p "$T/src/match" "$T/src/tools"
cp "$HERE/esa_linsmax.c" "$HERE/esa_linsmax.h" "$T/src/match/"
cp "$REF/src/tools/gt_repfind.c" "$T/src/tools/gt_repfind.c"
(cd "$T" && patch -s -p1 < "$HERE/gt_repfind_smax.patch")
CFLAGS="-std=c99 -Wall -Wextra -Wno-unused-parameter -Werror -D_GNU_SOURCE"
INC="-I$T/src -I$REF/src -I$ROOT/include"
gcc $CFLAGS $INC -c -o "$T/esa_linsmax.o" "$T/src/match/esa_linsmax.c"
gcc $CFLAGS $INC -c -o "$T/gt_repfind.o" "$T/src/tools/gt_repfind.c"
# the shim defines the runner's new entry point and binds the C-ABI
nm "$T/esa_linsmax.o" | grep -q " T gt_callenumsupermaxrepeats$"
nm "$T/esa_linsmax.o" | grep -q " U gt_smax_hip_enumerate$"
nm "$T/gt_repfind.o" | grep -q " U gt_callenumsupermaxrepeats$"
echo "shim + patched gt_repfind.c compile against $REF"

#!/bin/bash
# tools/probe/cold_probe.sh OUT -- a fresh process's first HIP stream against
# the device memory the previous process held (and whether it freed it or
# just exited) and the time since it exited.  One JSON object per line.
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
P=$R/tools/probe/cold_probe
OUT=$1
: > "$OUT"
run() { echo "{\"step\":\"$1\"}" >> "$OUT"; timeout -k 5 120 "$P" "${@:2}" >> "$OUT"; }
run "probe, idle device" probe
for GB in 0 8 32 96 192; do
  for MODE in free exit; do
    run "hold $GB GiB ($MODE)" hold "$GB" "$MODE"
    run "probe right after" probe
    run "probe again" probe
    sleep 2
    run "probe after 2 s" probe
  done
done

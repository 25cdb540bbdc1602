#!/usr/bin/env python3
"""Phase breakdown of the host-table entry point (gt_smax_hip_enumerate_to_buffer)
on C3: validate / H2D / plan / run / D2H+triples (GT_SMAX_TIMING=1 prints them
from the C-ABI layer), several calls in a row (the first pays one-time costs: pinned ring, device cache)."""
import os
import sys
import time

os.environ["GT_SMAX_TIMING"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402  (one HIP runtime per process: torch first)
import genometools_smax_amd as G  # noqa: E402

bases = int(float(sys.argv[1])) if len(sys.argv) > 1 else 3_000_000_000
text = G.synth_genome("human", bases, 1, threads=16)
esa = G.DeviceEsa(text, device=0, keep_suftab=False)
host = esa.download()
n, N = esa.totallength, esa.nonspecials
esa.release()
threads = [x for x in os.environ.get("THREADS_LIST", "").split(",") if x]
for i in range(int(os.environ.get("CALLS", "6"))):
    if threads:
        os.environ["GT_SMAX_COPY_THREADS"] = threads[i % len(threads)]
        print("GT_SMAX_COPY_THREADS=%s" % threads[i % len(threads)], file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    iv = G.enumerate_smax(host["lcptab"], host["llvtab"], host["bwttab"], n, N, 20, 1)
    print("call %d: %.1f ms, %d intervals" % (i, (time.perf_counter() - t0) * 1e3, len(iv)),
          file=sys.stderr, flush=True)
    del iv

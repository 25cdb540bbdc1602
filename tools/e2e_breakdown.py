#!/usr/bin/env python3
"""Phase breakdown of the host-table entry point (gt_smax_hip_enumerate_to_buffer)
on C3: validate / H2D / plan / run / D2H+triples (GT_SMAX_TIMING=1 prints them
from the C-ABI layer), several calls in a row (the first pays one-time costs: pinned ring, device cache).
SHARDS=W: num_gpus = W (on one device the W shards run one after another on
that device's thread: per-shard fill / H2D / plan / run phases); the records
of every call are compared with the oracle's."""
import os
import sys
import time

os.environ["GT_SMAX_TIMING"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: F401,E402  (one HIP runtime per process: torch first)
import genometools_smax_amd as G  # noqa: E402

bases = int(float(sys.argv[1])) if len(sys.argv) > 1 else 3_000_000_000
text = G.synth_genome("human", bases, 1, threads=16)
esa = G.DeviceEsa(text, device=0, keep_suftab=False)
host = esa.download()
n, N = esa.totallength, esa.nonspecials
esa.release()
threads = [x for x in os.environ.get("THREADS_LIST", "").split(",") if x]
shards = int(os.environ.get("SHARDS", "1"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib  # noqa: E402  (the checker)
want = oracle_lib.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], N, 20, threads=16)
for i in range(int(os.environ.get("CALLS", "6"))):
    if threads:
        os.environ["GT_SMAX_COPY_THREADS"] = threads[i % len(threads)]
        print("GT_SMAX_COPY_THREADS=%s" % threads[i % len(threads)], file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    iv = G.enumerate_smax(host["lcptab"], host["llvtab"], host["bwttab"], n, N, 20, shards)
    print("call %d (%d shards): %.1f ms, %d intervals, equal to the oracle: %s"
          % (i, shards, (time.perf_counter() - t0) * 1e3, len(iv), bool(np.array_equal(iv, want))),
          file=sys.stderr, flush=True)
    del iv

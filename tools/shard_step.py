#!/usr/bin/env python3
"""Diagnostic: the per-rank step of the W-GPU strong-scaling run, on one GPU:
one C3 ESA, then for each of W row shards (the bench's ownership rule) a
plan over rows [begin, end); prints step and K1 times (HIP events) -- the
local part of the step, without the RCCL exchange.  Args: kind bases minlen W"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import genometools_smax_amd as G  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "human"
bases = int(float(sys.argv[2])) if len(sys.argv) > 2 else 3_000_000_000
minlen = int(sys.argv[3]) if len(sys.argv) > 3 else 20
W = int(sys.argv[4]) if len(sys.argv) > 4 else 8
text = G.synth_genome(kind, bases, {"uniform": 42, "human": 1, "plant": 2}[kind])
esa = G.DeviceEsa(text)
del text
N = esa.nonspecials
s = torch.cuda.current_stream()
for r in range(W):
    begin = 1 + (N - 1) * r // W
    end = 1 + (N - 1) * (r + 1) // W
    p = esa.plan(minlen, begin, end)
    for _ in range(5):
        p.run(s.cuda_stream)
    # K1 from the plan's events around every K1 of one pass; the step from
    # a second pass without them (an event record between K1 and K1b costs
    # ~5.7 us, profiles/r04r/)
    p.enable_timing(50)
    for _ in range(50):
        p.run(s.cuda_stream)
    torch.cuda.synchronize()
    k1, n = p.kernel_ms()
    p.enable_timing(0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(50):
        p.run(s.cuda_stream)
    e1.record(s)
    torch.cuda.synchronize()
    st = e0.elapsed_time(e1) / 50
    print("shard %d/%d rows %d: step %.4f ms, K1 %.4f ms, rest %.4f ms, deferred %d"
          % (r, W, end - begin, st, k1 / n, st - k1 / n, p.deferred_tiles()), flush=True)
    p.close()

#!/usr/bin/env python3
"""Diagnostic: K1 time under ablation bits (GT_SMAX_DEBUG), one process,
interleaved rounds.  Outputs are wrong under ablation -- timing only.
bits: 1 skip look-back wait, 2 skip phase 1, 4 skip diversity, 8 skip writes."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import genometools_smax_amd as G
import torch

kind = sys.argv[1] if len(sys.argv) > 1 else "human"
bases = int(float(sys.argv[2])) if len(sys.argv) > 2 else 300_000_000
variants = [int(x, 0) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0, 1, 2, 4, 8, 15]
minlen = int(sys.argv[4]) if len(sys.argv) > 4 else 20
text = G.synth_genome(kind, bases, 1 if kind != "uniform" else 42)
esa = G.DeviceEsa(text)
print("n=%d N=%d llv=%d" % (esa.totallength, esa.nonspecials, esa.numllv), flush=True)
res = {v: [] for v in variants}
for rnd in range(3):
    for v in variants:
        os.environ["GT_SMAX_DEBUG"] = str(v)
        p = esa.plan(minlen)
        p.run(); torch.cuda.synchronize()
        if rnd == 0:
            print("dbg=%d: %d of %d tiles deferred to K1b" % (v, p.deferred_tiles(), p.num_tiles),
                  flush=True)
        if p.error_bits():
            print("dbg=%d: device error bits 0x%x" % (v, p.error_bits()), flush=True)
        p.enable_timing(10)
        for _ in range(10):
            p.run()
        ms, n = p.kernel_ms()
        res[v].append(ms / n)
        p.close()
for v in variants:
    print("dbg=%2d  K1 ms: min %.4f med %.4f" % (v, min(res[v]), sorted(res[v])[1]), flush=True)

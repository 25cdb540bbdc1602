#!/usr/bin/env python3
"""Diagnostic: K1 time versus persistent grid size (GT_SMAX_GRID), one
process, interleaved rounds."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import genometools_smax_amd as G
import torch

kind = sys.argv[1] if len(sys.argv) > 1 else "human"
bases = int(float(sys.argv[2])) if len(sys.argv) > 2 else 300_000_000
grids = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0, 768, 1024, 1280]
text = G.synth_genome(kind, bases, 1 if kind != "uniform" else 42)
esa = G.DeviceEsa(text)
os.environ["GT_SMAX_VERBOSE"] = "1"
res = {g: [] for g in grids}
for rnd in range(3):
    for g in grids:
        os.environ["GT_SMAX_GRID"] = str(g)
        p = esa.plan(20)
        p.run(); torch.cuda.synchronize()
        p.enable_timing(10)
        for _ in range(10):
            p.run()
        ms, n = p.kernel_ms()
        res[g].append(ms / n)
        p.close()
    os.environ.pop("GT_SMAX_VERBOSE", None)
for g in grids:
    print("grid=%5d  K1 ms: min %.4f med %.4f" % (g, min(res[g]), sorted(res[g])[1]), flush=True)

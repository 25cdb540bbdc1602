#!/usr/bin/env python3
"""Diagnostic: why K1 defers tiles to K1b on a workload -- tiles whose .llv
window exceeds K1's staged values (SMAX_LLV_CAP), shard-edge tiles, and the
rest (exact-queue overflow).  Timing only for the run itself."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import genometools_smax_amd as G

kind = sys.argv[1] if len(sys.argv) > 1 else "human"
bases = int(float(sys.argv[2])) if len(sys.argv) > 2 else 300_000_000
cap = int(sys.argv[3]) if len(sys.argv) > 3 else 112
TILE, H = 2048, 16
text = G.synth_genome(kind, bases, 1 if kind != "uniform" else 42)
esa = G.DeviceEsa(text)
p = esa.plan(20)
p.run()
torch.cuda.synchronize()
nd = p.deferred_tiles()
pos = esa.download()["llvtab"][:, 0].astype(np.int64)
N = esa.nonspecials
nt = p.num_tiles
g0 = np.arange(nt, dtype=np.int64) * TILE
lo = np.searchsorted(pos, np.maximum(g0 - H, 0))
hi = np.searchsorted(pos, g0 + TILE + H)
wn = hi - lo
print("N=%d tiles=%d deferred=%d llv=%d" % (N, nt, nd, len(pos)))
for c in (64, 112, 128, 160, 224, 256, 512, 1024):
    print("  tiles with > %4d .llv in window: %d" % (c, int(np.count_nonzero(wn > c))))
print("  tiles with any .llv: %d; max per window %d" % (int(np.count_nonzero(wn)), int(wn.max())))

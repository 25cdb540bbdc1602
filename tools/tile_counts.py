#!/usr/bin/env python3
"""Diagnostic: distribution of smax records per 2048-row tile (slot sizing)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch  # noqa: F401
import genometools_smax_amd as G

kind = sys.argv[1] if len(sys.argv) > 1 else "human"
bases = int(float(sys.argv[2])) if len(sys.argv) > 2 else 3_000_000_000
minlen = int(sys.argv[3]) if len(sys.argv) > 3 else 20
text = G.synth_genome(kind, bases, {"uniform": 42, "human": 1, "plant": 2}[kind])
esa = G.DeviceEsa64(text) if len(text) + 1 >= 2 ** 32 else G.DeviceEsa(text)
del text
p = esa.plan(minlen)
p.run()
torch.cuda.synchronize()
counts, _ = p.debug_tiles()
print("%s %.3g bp minlen %d: %d tiles, %d records" % (kind, bases, minlen, len(counts), counts.sum()))
for c in (8, 16, 32, 48, 64, 96, 128, 192, 256, 512):
    m = counts > c
    print("  tiles with > %3d records: %8d (%.3f%%), holding %d records"
          % (c, m.sum(), 100.0 * m.mean(), counts[m].sum()))
print("  max %d" % counts.max())

#!/usr/bin/env python3
"""Diagnostic: per-tile K1b cost (GT_SMAX_DEBUG=32768 cycle stamps) of the
deferred tiles on a synthetic genome, with their LCP-window statistics."""
import os
import sys

os.environ["GT_SMAX_DEBUG"] = str(32768 | int(os.environ.get("EXTRA_DBG", "0")))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import genometools_smax_amd as G

kind = sys.argv[1] if len(sys.argv) > 1 else "human"
bases = int(float(sys.argv[2])) if len(sys.argv) > 2 else 300_000_000
text = G.synth_genome(kind, bases, 1 if kind != "uniform" else 42)
esa = G.DeviceEsa(text)
p = esa.plan(20)
p.run()
torch.cuda.synchronize()
counts, deferred = p.debug_tiles()
d = esa.download()
L = d["lcptab"]
cyc = (counts[deferred] & 0x7fffffff).astype(np.int64) * 16
gen = (counts[deferred] >> 31).astype(bool)
print("deferred %d tiles; K1b cycles per tile: sum %.3g mean %.0f p50 %.0f p90 %.0f p99 %.0f max %.0f; generic path %d"
      % (len(deferred), cyc.sum(), cyc.mean(), np.percentile(cyc, 50), np.percentile(cyc, 90),
         np.percentile(cyc, 99), cyc.max(), gen.sum()))
order = np.argsort(-cyc)[:15]
for i in order:
    t = int(deferred[i])
    w = L[t * 2048: t * 2048 + 2048].astype(np.int32)
    ff = int((w == 255).sum())
    eq = np.concatenate(([False], (w[1:] == w[:-1]) & (w[1:] >= 20)))
    # longest run of equal bytes >= 20
    best = run = 0
    for e in eq:
        run = run + 1 if e else 0
        best = max(best, run)
    print("  tile %8d: %9d cycles generic=%d  255-bytes %4d  longest equal run %4d  max byte %d"
          % (t, cyc[i], gen[i], ff, best, w.max()))

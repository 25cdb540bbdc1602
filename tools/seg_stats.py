#!/usr/bin/env python3
"""Diagnostic: K1's per-tile segment statistics on a sample of tiles --
active segments (a byte >= min(minlen,128)), those left by the start filter
(LCP >= mf with BWT[c-1] != BWT[c] or special, or a 255 byte), and how many
tiles need a second 64-lane classification step.  Args: kind bases minlen."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import genometools_smax_amd as G  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "human"
bases = int(float(sys.argv[2])) if len(sys.argv) > 2 else 3_000_000_000
minlen = int(sys.argv[3]) if len(sys.argv) > 3 else 20
text = G.synth_genome(kind, bases, 1 if kind != "uniform" else 42)
esa = G.DeviceEsa(text)
del text
d = esa.download()
lcp, bwt = d["lcptab"], d["bwttab"]
esa.release()
mf = min(minlen, 128)
T = 2048
ntiles = (len(lcp) - 1) // T
rng = np.random.default_rng(0)
sample = np.sort(rng.choice(ntiles - 2, size=min(20000, ntiles - 2), replace=False) + 1)
act, filt = [], []
for t in sample:
    g0 = t * T
    L = lcp[g0:g0 + T].reshape(128, 16)
    B = bwt[g0 - 1:g0 + T].astype(np.int32)
    a = (L >= mf).any(axis=1)
    div = (B[1:] != B[:-1]) | (B[1:] >= 254) | (B[:-1] >= 254)
    cs = ((L.reshape(-1) >= mf) & div).reshape(128, 16).any(axis=1) | (L == 255).any(axis=1)
    act.append(int(a.sum()))
    filt.append(int((a & cs).sum()))
act, filt = np.array(act), np.array(filt)
print("%s %.1e minlen %d: %d tiles sampled" % (kind, bases, minlen, len(sample)))
print("active segments/tile: mean %.1f, p50 %d, p90 %d, >64: %.1f%%" %
      (act.mean(), np.median(act), np.percentile(act, 90), 100 * (act > 64).mean()))
print("after start filter:   mean %.1f, >64: %.1f%% (two classification steps)" %
      (filt.mean(), 100 * ((act > 64) & (filt > 64)).mean()))
print("tiles with no active segment: %.1f%%" % (100 * (act == 0).mean()))

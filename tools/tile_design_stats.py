#!/usr/bin/env python3
"""Diagnostic: how many 64-lane classification steps K1 would need per tile
under different segment filters and tile sizes (a sample of tiles of the
GPU-built ESA).  Filters of a 16-row segment:
  any    a byte >= mf (mf = min(minlen, 128))                 -- K1's first filter
  div    a row c with LCP[c] >= mf and BWT[c-1] != BWT[c] (or a special), or
         a 255 byte                                           -- K1's refinement
  start  a row c with LCP[c] >= mf, LCP[c] > LCP[c-1] (255 after 255 counted
         as possible) and BWT[c-1] != BWT[c] (or special), or a 255 byte:
         the rows that can start a record at all
and the same at 4-row word granularity.  Args: kind bases minlen."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import genometools_smax_amd as G  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "human"
bases = int(float(sys.argv[2])) if len(sys.argv) > 2 else 3_000_000_000
minlen = int(sys.argv[3]) if len(sys.argv) > 3 else 20
text = G.synth_genome(kind, bases, {"uniform": 42, "plant": 2}.get(kind, 1), threads=16)
esa = G.DeviceEsa64(text) if len(text) + 1 >= 2 ** 32 else G.DeviceEsa(text)
del text
d = esa.download()
lcp, bwt = d["lcptab"], d["bwttab"]
esa.release()
mf = min(minlen, 128)
T = 4096
ntiles = (len(lcp) - 1) // T
rng = np.random.default_rng(0)
sample = np.sort(rng.choice(ntiles - 2, size=min(20000, ntiles - 2), replace=False) + 1)
res = {k: {2048: [], 4096: []} for k in ("any", "div", "start", "w_any", "w_start", "rows_start")}
for t in sample:
    g0 = t * T
    L = lcp[g0 - 1:g0 + T].astype(np.int32)
    B = bwt[g0 - 1:g0 + T].astype(np.int32)
    c, p = L[1:], L[:-1]
    ge = c >= mf
    ff = c == 255
    div = (B[1:] != B[:-1]) | (B[1:] >= 254) | (B[:-1] >= 254)
    up = (c > p) | (ff & (p == 255))
    st = (ge & up & div) | ff
    dv = (ge & div) | ff
    for half in (2048, 4096):
        for h0 in range(0, T, half):
            sl = slice(h0, h0 + half)
            res["any"][half].append(int(ge[sl].reshape(-1, 16).any(1).sum()))
            res["div"][half].append(int(dv[sl].reshape(-1, 16).any(1).sum()))
            res["start"][half].append(int(st[sl].reshape(-1, 16).any(1).sum()))
            res["w_any"][half].append(int(ge[sl].reshape(-1, 4).any(1).sum()))
            res["w_start"][half].append(int(st[sl].reshape(-1, 4).any(1).sum()))
            res["rows_start"][half].append(int(st[sl].sum()))
print("%s %.2e minlen %d: %d tiles of 4096 sampled" % (kind, bases, minlen, len(sample)))
for half in (2048, 4096):
    segs = half // 16
    print("-- tile %d rows (%d segments, %d words)" % (half, segs, half // 4))
    for k, v in res.items():
        a = np.array(v[half])
        unit = 64 if not k.startswith("w_") else 256   # 64 lanes x 4 words
        steps = np.maximum(1, (a + unit - 1) // unit) if k != "rows_start" else None
        line = "%-10s mean %7.1f p50 %5d p90 %5d p99 %5d" % (k, a.mean(), np.percentile(a, 50),
                                                           np.percentile(a, 90), np.percentile(a, 99))
        if steps is not None:
            line += "  steps/tile mean %.3f (>1: %.1f%%)" % (steps.mean(), 100 * (steps > 1).mean())
        print(line)

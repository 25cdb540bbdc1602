#!/usr/bin/env python3
"""Diagnostic: workload statistics of the K1 detection path on a synthetic
genome (GPU ESA, downloaded; numpy on the host).  Prints how many rows pass
each filter stage, the plateau-start density per 1024-row wave round and
the share of starts that leave the fast (<= 7-row plateau, byte) path."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import genometools_smax_amd as G

kind = sys.argv[1] if len(sys.argv) > 1 else "human"
bases = int(float(sys.argv[2])) if len(sys.argv) > 2 else 300_000_000
minlen = int(sys.argv[3]) if len(sys.argv) > 3 else 20
text = G.synth_genome(kind, bases, 1 if kind != "uniform" else 42)
esa = G.DeviceEsa(text)
d = esa.download()
L = np.asarray(d["lcptab"], dtype=np.uint8)
N = esa.nonspecials
L = L[: N + 1].astype(np.int16)
rows = N + 1
print("rows %d  llv %d" % (rows, esa.numllv))
ge = L >= minlen
print("LCP>=minlen: %.3f" % ge.mean())
prev = np.concatenate(([0], L[:-1]))
start = ge & (L > prev)
print("plateau starts: %d (%.4f of rows)" % (start.sum(), start.mean()))
seg = rows // 16
segge = ge[: seg * 16].reshape(seg, 16).any(1)
print("16-row segments passing the filter: %.3f" % segge.mean())
rnd = rows // 1024
per = start[: rnd * 1024].reshape(rnd, 1024).sum(1)
print("starts per 1024-row round: mean %.1f  p50 %d  p90 %d  p99 %d  max %d" %
      (per.mean(), np.percentile(per, 50), np.percentile(per, 90), np.percentile(per, 99), per.max()))
steps = np.ceil(per / 64)
print("64-start evaluation steps per round: mean %.2f  (rounds with 0: %.3f)" %
      (steps.mean(), (per == 0).mean()))
idx = np.nonzero(start)[0]
cb255 = (L[idx] == 255).mean()
# plateau length from each start
nxt = np.ones(len(idx), dtype=np.int64)
eq = np.zeros(len(idx), dtype=bool)
for k in range(1, 9):
    j = np.minimum(idx + k, rows - 1)
    same = L[j] == L[idx]
    if k == 1:
        eq = same
    else:
        eq &= same
    nxt += eq
print("starts with a 255 byte: %.4f   plateaus > 7 rows: %.4f" % (cb255, (nxt > 7).mean()))
lm = np.zeros(len(idx), dtype=bool)
endj = np.minimum(idx + nxt, rows - 1)
lm = L[endj] < L[idx]
print("local maxima among starts: %.3f  (width mean %.2f)" % (lm.mean(), (nxt[lm] + 1).mean()))
nxt1 = L[np.minimum(idx + 1, rows - 1)]
eqn = nxt1 == L[idx]
ffs = L[idx] == 255
print("starts with LCP[c+1]==LCP[c]: %.3f   with 255 byte: %.3f   -> exact queue %.3f" %
      (eqn.mean(), ffs.mean(), (eqn | ffs).mean()))
per_tile = np.bincount((idx[eqn | ffs] // 2048), minlength=rows // 2048 + 1)
print("exact-queue starts per 2048-row tile: mean %.1f p50 %d p90 %d p99 %d max %d; tiles > 64: %.4f" %
      (per_tile.mean(), np.percentile(per_tile, 50), np.percentile(per_tile, 90),
       np.percentile(per_tile, 99), per_tile.max(), (per_tile > 64).mean()))
# plateau length (rows) of the exact-queue starts
eqi = idx[eqn & ~ffs]
plen = np.ones(len(eqi), dtype=np.int64)
alive = np.ones(len(eqi), dtype=bool)
for k in range(1, 16):
    j = np.minimum(eqi + k, rows - 1)
    alive &= L[j] == L[eqi]
    plen += alive
print("plateau rows of LCP[c+1]==LCP[c] starts: 2: %.3f  3: %.3f  4-7: %.3f  8+: %.3f" %
      ((plen == 2).mean(), (plen == 3).mean(), ((plen >= 4) & (plen <= 7)).mean(), (plen >= 8).mean()))
# active 16-row segments per 2048-row tile (K1 classification steps of 64)
nt = rows // 2048
act = segge[: nt * 128].reshape(nt, 128).sum(1)
print("active segments per tile: mean %.1f p10 %d p50 %d p90 %d; tiles needing 2 steps: %.3f, 0 steps: %.3f"
      % (act.mean(), np.percentile(act, 10), np.percentile(act, 50), np.percentile(act, 90),
         (act > 64).mean(), (act == 0).mean()))
print("histogram of active segments per tile (bins of 16):",
      np.bincount(np.minimum(act // 16, 8), minlength=9).tolist())

#!/usr/bin/env python3
"""Diagnostic: per K1 tile (2048 rows) of one bench config, how many of its
128 16-row segments pass the filter (some LCP byte >= min(minlen, 128)) and
how many smax records it holds -- the work K1 does beyond the window
stream.

  tile_stats.py CONFIG        (bench.py config: c2, c3, c5 ...)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import genometools_smax_amd as G  # noqa: E402

TILE, SEG = 2048, 16
cfg = bench.CONFIGS[sys.argv[1]]
minlen = cfg["minlen"]
text = G.synth_genome(cfg["kind"], cfg["bases"], cfg["seed"], threads=16)
n = len(text)
esa = G.DeviceEsa64(text, device=0) if n + 1 >= 2 ** 32 else G.DeviceEsa(text, device=0)
del text
N = esa.nonspecials
plan = esa.plan(minlen)
plan.run()
trip = plan.fetch_triples()
plan.close()
dl = esa.download()
lcp, bwt = dl["lcptab"], dl["bwttab"]
del dl
esa.release()
ntiles = (N + TILE - 1) // TILE
mf = min(minlen, 128)
act = np.zeros(ntiles, dtype=np.int32)
# classification steps of 64 segments: K1 filters segments further when more
# than 64 are active (prepare_window): "can" keeps those with a row c of LCP
# >= mf whose BWT differs from row c-1's (or is special) or with a 255 byte;
# "up" additionally needs LCP[c] > LCP[c-1] (a record start's condition)
steps = {"ge": np.zeros(ntiles, np.int8), "can": np.zeros(ntiles, np.int8),
         "up": np.zeros(ntiles, np.int8)}
# LCP chunks of 32 / 64 / 128 bytes with no byte >= mf (a zone map per 16
# rows would let K1 skip their DMA), and runs of such chunks
idle = {32: 0, 64: 0, 128: 0}
CH = 1 << 16                      # tiles per chunk
for t0 in range(0, ntiles, CH):
    t1 = min(ntiles, t0 + CH)
    seg = lcp[t0 * TILE: t1 * TILE]
    pad = (t1 - t0) * TILE - len(seg)
    if pad:
        seg = np.concatenate([seg, np.zeros(pad, np.uint8)])
    a16 = (seg.reshape(t1 - t0, TILE // SEG, SEG) >= mf).any(axis=2)
    act[t0:t1] = a16.sum(axis=1)
    r0, r1 = t0 * TILE, t0 * TILE + len(seg) - pad
    b = bwt[r0:r1]
    bp = np.concatenate([bwt[r0 - 1:r0] if r0 else np.zeros(1, np.uint8), b[:-1]])
    lp = np.concatenate([lcp[r0 - 1:r0] if r0 else np.zeros(1, np.uint8), seg[:len(b) - 1]])
    ge = seg[:len(b)] >= mf
    div = (b != bp) | (b >= 4) | (bp >= 4)
    ff = seg[:len(b)] == 255
    can = (ge & div) | ff
    up = (ge & div & (seg[:len(b)] > lp)) | ff
    del b, bp, div
    for key, m in (("can", can), ("up", up)):
        if pad:
            m = np.concatenate([m, np.zeros(pad, bool)])
        n = m.reshape(t1 - t0, TILE // SEG, SEG).any(axis=2).sum(axis=1)
        n = np.where(act[t0:t1] > 64, n, act[t0:t1])
        steps[key][t0:t1] = (n + 63) // 64
    steps["ge"][t0:t1] = (act[t0:t1] + 63) // 64
    del ge, ff, can, up, lp
    for w in idle:
        idle[w] += int((~a16.reshape(t1 - t0, -1, w // SEG).any(axis=2)).sum())
rec = np.bincount((trip[:, 1] // TILE).astype(np.int64), minlength=ntiles)[:ntiles]
print("%s: N=%d, %d tiles, %d records (%.2f per tile)" % (sys.argv[1], N, ntiles, len(trip),
                                                          len(trip) / ntiles))
print("active segments per tile (of 128): mean %.1f" % act.mean())
for lo, hi in ((0, 0), (1, 16), (17, 32), (33, 64), (65, 96), (97, 128)):
    m = (act >= lo) & (act <= hi)
    print("  %3d-%3d: %6.2f %% of tiles" % (lo, hi, 100.0 * m.mean()))
for key, lab in (("ge", "LCP >= mf only"), ("can", "K1's filter (>= mf, BWT differs, or 255)"),
                 ("up", "+ LCP[c] > LCP[c-1]")):
    st = steps[key]
    print("classification steps per tile, %s: mean %.3f, 2 steps in %.2f %% of tiles" %
          (lab, st.mean(), 100.0 * (st >= 2).mean()))
for w in sorted(idle):
    tot = ntiles * TILE // w
    print("LCP chunks of %3d B with no byte >= %d: %6.2f %%" % (w, mf, 100.0 * idle[w] / tot))
print("records per tile: max %d" % rec.max())
for lo, hi in ((0, 0), (1, 8), (9, 16), (17, 32), (33, 64), (65, 1 << 30)):
    m = (rec >= lo) & (rec <= hi)
    print("  %3d-%s: %6.2f %% of tiles" % (lo, hi if hi < 1 << 30 else "", 100.0 * m.mean()))

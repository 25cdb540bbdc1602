#!/usr/bin/env python3
"""Diagnostic: .llv entries per K1 tile window (rows [g0-16, g0+2048+16) of
every 2048-row tile) for one bench config, and how many tiles a given LDS
cap on the staged values would leave to the static K1b list.

  llv_window_stats.py CONFIG        (bench.py config: c2, c3, c5 ...)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import genometools_smax_amd as G  # noqa: E402

TILE, HALO = 2048, 16
cfg = bench.CONFIGS[sys.argv[1]]
text = G.synth_genome(cfg["kind"], cfg["bases"], cfg["seed"], threads=16)
n = len(text)
esa = G.DeviceEsa64(text, device=0) if n + 1 >= 2 ** 32 else G.DeviceEsa(text, device=0)
del text
N = esa.nonspecials
pos = esa.download()["llvtab"][:, 0].astype(np.int64) if esa.numllv else np.zeros(0, np.int64)
esa.release()
ntiles = (N + TILE - 1) // TILE
starts = np.arange(ntiles, dtype=np.int64) * TILE
lo = np.searchsorted(pos, starts - HALO)
hi = np.searchsorted(pos, starts + TILE + HALO)
cnt = hi - lo
print("%s: N=%d, %d tiles, %d .llv entries, mean %.2f per window, max %d"
      % (sys.argv[1], N, ntiles, len(pos), cnt.mean(), cnt.max()))
for cap in (64, 96, 128, 160, 192, 224, 240, 256, 320, 384, 496):
    m = cnt > cap
    print("  windows with > %3d values: %8d (%.4f%% of tiles)" % (cap, m.sum(), 100.0 * m.mean()))

#!/usr/bin/env python3
"""Diagnostic: where K1's wave time goes, per tile, from s_memtime stamps in
the diagnostic build (GT_SMAX_STAMPS; gt_smax_plan_stamps): window wait,
flush + next DMA issue, segment filter, classification + exact queue,
exact starts, record output, staging.  The cycles are wave cycles (a wave's
wall time per section, its SIMD shared by the other resident waves), so
they add up to the time a wave spends per tile.  Args: config [runs]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import genometools_smax_amd as G  # noqa: E402
import torch  # noqa: E402

cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
runs = int(sys.argv[2]) if len(sys.argv) > 2 else 5
text = G.synth_genome(cfg["kind"], cfg["bases"], cfg["seed"], threads=16)
esa = G.DeviceEsa64(text, device=0) if len(text) + 1 >= 2 ** 32 else G.DeviceEsa(text, device=0)
del text
L = G.lib()
L.gt_smax_plan_stamps.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong)]
plain = esa.plan(cfg["minlen"])
os.environ["GT_SMAX_STAMPS"] = "1"
p = esa.plan(cfg["minlen"])
os.environ.pop("GT_SMAX_STAMPS")
for q, name in ((plain, "production"), (p, "stamped diag")):
    q.enable_timing(runs)
    for _ in range(runs):
        q.run()
    torch.cuda.synchronize()
    ms, n = q.kernel_ms()
    print("K1 %s: %.4f ms" % (name, ms / max(n, 1)), flush=True)
out = (ctypes.c_ulonglong * 8)()
assert L.gt_smax_plan_stamps(p.plan, out) == 0
tiles = out[7]
names = ["window wait", "flush + next DMA issue", "segment filter", "classify + exact queue",
         "exact starts", "record output", "staging move"]
tot = sum(out[k] for k in range(7))
print("tiles %d (%d runs); wave cycles per tile:" % (tiles, runs))
for k in range(7):
    print("  %-24s %8.0f  (%4.1f %%)" % (names[k], out[k] / tiles, 100.0 * out[k] / tot))
print("  %-24s %8.0f" % ("total", tot / tiles))

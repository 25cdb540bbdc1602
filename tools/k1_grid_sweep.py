#!/usr/bin/env python3
"""Diagnostic: K1 grid (GT_SMAX_GRID workgroups) vs step and K1 time (HIP
events) on one shard of a W-way split.  Args: kind bases minlen shard/of grids..."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import genometools_smax_amd as G  # noqa: E402

kind, bases, minlen = sys.argv[1], int(float(sys.argv[2])), int(sys.argv[3])
si, sw = (int(x) for x in sys.argv[4].split("/"))
grids = [int(x) for x in sys.argv[5:]]
text = G.synth_genome(kind, bases, {"uniform": 42, "human": 1, "plant": 2}[kind])
esa = G.DeviceEsa(text)
del text
N = esa.nonspecials
begin, end = 1 + (N - 1) * si // sw, 1 + (N - 1) * (si + 1) // sw
s = torch.cuda.current_stream()
sp = s.cuda_stream
L = G.lib()
plans = {}
for g in grids:
    os.environ["GT_SMAX_GRID"] = str(g)
    plans[g] = esa.plan(minlen, begin, end)
os.environ.pop("GT_SMAX_GRID", None)
res = {g: [] for g in grids}
for rnd in range(5):
    for g in (grids if rnd % 2 == 0 else grids[::-1]):
        p = plans[g]
        for _ in range(3):
            p.run(sp)
        p.enable_timing(30)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(30):
            p.run(sp)
        e1.record(s)
        torch.cuda.synchronize()
        k1, n = p.kernel_ms()
        res[g].append((e0.elapsed_time(e1) / 30, k1 / max(n, 1)))
print("rows [%d, %d) (shard %d/%d), %d tiles" % (begin, end, si, sw, plans[grids[0]].num_tiles))
for g in grids:
    st = sorted(x[0] for x in res[g])
    k = sorted(x[1] for x in res[g])
    print("grid %6d: step %.4f ms  K1 %.4f ms (medians of 5)" % (g, st[2], k[2]), flush=True)

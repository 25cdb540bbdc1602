#!/usr/bin/env python3
"""Diagnostic: cost of bench.py's per-step K1 HIP events (gt_smax_plan_timing)
on the step, interleaved with and without them on one plan.
Args: kind bases minlen shard/of"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import genometools_smax_amd as G  # noqa: E402

kind, bases, minlen = sys.argv[1], int(float(sys.argv[2])), int(sys.argv[3])
si, sw = (int(x) for x in sys.argv[4].split("/"))
text = G.synth_genome(kind, bases, {"uniform": 42, "human": 1, "plant": 2}[kind])
esa = G.DeviceEsa(text)
del text
N = esa.nonspecials
begin, end = 1 + (N - 1) * si // sw, 1 + (N - 1) * (si + 1) // sw
s = torch.cuda.current_stream()
sp = s.cuda_stream
p = esa.plan(minlen, begin, end)
res = {True: [], False: []}
for rnd in range(8):
    for ev in ((True, False) if rnd % 2 == 0 else (False, True)):
        for _ in range(3):
            p.run(sp)
        p.enable_timing(50 if ev else 0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(s)
        for _ in range(50):
            p.run(sp)
        e1.record(s)
        torch.cuda.synchronize()
        res[ev].append(e0.elapsed_time(e1) / 50)
a, b = sorted(res[True]), sorted(res[False])
print("rows [%d, %d) (shard %d/%d): step with K1 events %.4f ms, without %.4f ms (medians of 8)"
      % (begin, end, si, sw, a[4], b[4]))

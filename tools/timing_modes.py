#!/usr/bin/env python3
"""Diagnostic: one plan over the C3 tables timed the way bench.py times it
(K1 HIP events on every 4th run, 50 runs, step time by host clock around
synchronisations) and the way tools/ab_interleave.py does (events on every
run, 30 runs, step time by torch events), alternated in rounds in one
process.  Separates a difference between the two tools' numbers from the
box and its state.  Args: kind bases minlen [rounds]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import genometools_smax_amd as G  # noqa: E402

kind, bases, minlen = sys.argv[1], int(float(sys.argv[2])), int(sys.argv[3])
rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 4
text = G.synth_genome(kind, bases, {"uniform": 42, "human": 1, "plant": 2}[kind], threads=16)
esa = G.DeviceEsa(text, keep_suftab=False)
del text
N = esa.nonspecials
p = esa.plan(minlen, 1, N)
s = torch.cuda.current_stream()
sp = s.cuda_stream


def bench_style(n=50, stride=4):
    for _ in range(5):
        p.run(sp)
    p.enable_timing((n + stride - 1) // stride, stride)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        p.run(sp)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) * 1e3 / n
    ms, k = p.kernel_ms()
    return el, ms / max(k, 1)


def ab_style(n=30):
    for _ in range(3):
        p.run(sp)
    p.enable_timing(n, 1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(n):
        p.run(sp)
    e1.record(s)
    torch.cuda.synchronize()
    ms, k = p.kernel_ms()
    return e0.elapsed_time(e1) / n, ms / max(k, 1)


# per-step times of the first passes of a fresh plan (torch events around
# each run): the shape of the warm-up transient
if len(sys.argv) > 5:
    q = p
    n = int(sys.argv[5])
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record(s)
        q.run(sp)
        e1.record(s)
    torch.cuda.synchronize()
    ts = [e0.elapsed_time(e1) for e0, e1 in evs]
    print("first %d passes of the plan after the ESA build (ms): %s" % (n, " ".join("%.3f" % x for x in ts)))
    time.sleep(2.0)
    for e0, e1 in evs[:40]:
        e0.record(s)
        q.run(sp)
        e1.record(s)
    torch.cuda.synchronize()
    print("after 2 s idle, 40 passes (ms): %s" % " ".join("%.3f" % e0.elapsed_time(e1) for e0, e1 in evs[:40]))


for r in range(rounds):
    a = bench_style()
    b = ab_style()
    c = bench_style(50, 1)
    print("round %d: bench-style step %.4f K1 %.4f | ab-style step %.4f K1 %.4f | "
          "bench-style, events every run: step %.4f K1 %.4f" % (r, a[0], a[1], b[0], b[1], c[0], c[1]),
          flush=True)
p.close()


#!/usr/bin/env python3
"""Diagnostic A/B/C/...: several builds of the library in ONE process on the
same device tables (the in-tree build first, then each LIB given), plans
created by each, runs rotated in rounds so that clock and thermal drift hit
all alike.  Prints per-build median step and K1 time (HIP events) and
whether each build's records equal the first's.

  ab_multi.py KIND BASES MINLEN SHARD ROUNDS LIB [LIB ...]
  (SHARD = i/w: plans over one shard's rows of the w-way split; a LIB path's
  parent directory names the build in the output)"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import genometools_smax_amd as G  # noqa: E402

kind, bases, minlen = sys.argv[1], int(float(sys.argv[2])), int(sys.argv[3])
si, sw = (int(x) for x in sys.argv[4].split("/"))
rounds = int(sys.argv[5])
# a LIB argument "shift:S" is the in-tree build over a copy of the LCP table
# placed so that its device address is S mod 128 (window-stream alignment)
args = sys.argv[6:]
paths = [G.LIB_PATH] + [G.LIB_PATH if a.startswith("shift:") else a for a in args]
names = ["in-tree"] + [a if a.startswith("shift:") else os.path.basename(os.path.dirname(a))
                       for a in args]
shifts = [None] + [int(a.split(":")[1]) if a.startswith("shift:") else None for a in args]
libs = []
for p in paths:
    G._lib, G.LIB_PATH = None, p
    libs.append(G.lib())
G._lib, G.LIB_PATH = libs[0], paths[0]

text = G.synth_genome(kind, bases, {"uniform": 42, "human": 1, "plant": 2}[kind])
esa = G.DeviceEsa(text) if len(text) + 1 < 2 ** 32 else G.DeviceEsa64(text)
del text
N = esa.nonspecials
begin, end = 1 + (N - 1) * si // sw, 1 + (N - 1) * (si + 1) // sw
print("rows [%d, %d) (shard %d/%d), builds: %s" % (begin, end, si, sw, ", ".join(names)), flush=True)
print("LCP table at %d mod 128" % (esa.esa.lcptab_dev % 128), flush=True)
plans = []
copies = []
for L, sh in zip(libs, shifts):
    G._lib = L
    if sh is None:
        plans.append(esa.plan(minlen, begin, end))
        continue
    n1 = esa.totallength + 1
    buf = torch.zeros(G.PAD_FRONT + n1 + G.PAD_BACK + 256, dtype=torch.uint8, device="cuda")
    off = G.PAD_FRONT + ((sh - (buf.data_ptr() + G.PAD_FRONT)) % 128)
    torch.cuda.synchronize()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy(ctypes.c_void_p(buf.data_ptr() + off), ctypes.c_void_p(esa.esa.lcptab_dev),
                  ctypes.c_size_t(n1), 3)   # hipMemcpyDeviceToDevice
    copies.append(buf)
    plans.append(G.SmaxPlan(buf.data_ptr() + off, esa.esa.bwttab_dev, esa.esa.llvtab_dev, esa.numllv,
                            0, n1, begin, end, N, minlen, esa.device, 0,
                            bwtpk_ptr=esa.esa.bwtpk_dev))
G._lib = libs[0]
s = torch.cuda.current_stream()
sp = s.cuda_stream
step = {n: [] for n in names}
k1 = {n: [] for n in names}


def timed(L, p, n=30):
    """(step, K1) in ms: K1 from the plan's own events around every K1 of a
    first pass; the step from a second pass with those events off (an event
    record between K1 and K1b costs ~5.7 us on the box, profiles/r04r/)."""
    for _ in range(3):
        L.gt_smax_plan_run(p.plan, sp)
    L.gt_smax_plan_timing(p.plan, n)
    for _ in range(n):
        L.gt_smax_plan_run(p.plan, sp)
    torch.cuda.synchronize()
    ms, k = ctypes.c_double(), ctypes.c_int()
    L.gt_smax_plan_timing_read(p.plan, ctypes.byref(ms), ctypes.byref(k))
    L.gt_smax_plan_timing(p.plan, 0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(n):
        L.gt_smax_plan_run(p.plan, sp)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n, ms.value / max(k.value, 1)


m = len(libs)
for r in range(rounds):
    order = [(r + j) % m for j in range(m)]          # rotate who goes first
    line = []
    for j in order:
        a, b = timed(libs[j], plans[j])
        step[names[j]].append(a)
        k1[names[j]].append(b)
        line.append("%s %.4f" % (names[j], a))
    print("round %d: %s" % (r, "  ".join(line)), flush=True)


def med(x):
    x = sorted(x)
    return x[len(x) // 2]


base = med(step[names[0]])
for j, n in enumerate(names):
    print("median %-12s step %.4f ms (x%.4f of %s)  K1 %.4f ms  rest %.4f ms"
          % (n, med(step[n]), med(step[n]) / base, names[0], med(k1[n]), med(step[n]) - med(k1[n])),
          flush=True)
G._lib = libs[0]
want = plans[0].fetch_triples()
for j in range(1, m):
    G._lib = libs[j]
    got = plans[j].fetch_triples()
    print("records %s == %s: %s (%d / %d)" % (names[j], names[0], bool((got == want).all())
                                              if got.shape == want.shape else False, len(got), len(want)),
          flush=True)
for j, p in enumerate(plans):
    G._lib = libs[j]
    p.close()
G._lib = libs[0]
esa.release()

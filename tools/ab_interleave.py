#!/usr/bin/env python3
"""Diagnostic A/B with the two builds in ONE process on the same device
tables: the in-tree library (A) and a second copy (B, path in argv[4]),
plans created by each, runs alternated in rounds so that clock and
thermal drift hit both alike.  Prints per-round and median step times.
Args: kind bases minlen libB [rounds] [shard/of: plans over one shard's rows]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import genometools_smax_amd as G  # noqa: E402

kind, bases, minlen, libb = sys.argv[1], int(float(sys.argv[2])), int(sys.argv[3]), sys.argv[4]
rounds = int(sys.argv[5]) if len(sys.argv) > 5 else 8
shard = sys.argv[6] if len(sys.argv) > 6 else "0/1"
si, sw = (int(x) for x in shard.split("/"))
LA = G.lib()
pa_path = G.LIB_PATH
G._lib, G.LIB_PATH = None, libb
LB = G.lib()
G._lib, G.LIB_PATH = LA, pa_path

text = G.synth_genome(kind, bases, {"uniform": 42, "human": 1, "plant": 2}[kind])
esa = G.DeviceEsa(text) if len(text) + 1 < 2 ** 32 else G.DeviceEsa64(text)
del text
N = esa.nonspecials
begin, end = 1 + (N - 1) * si // sw, 1 + (N - 1) * (si + 1) // sw
print("rows [%d, %d) (shard %d/%d)" % (begin, end, si, sw), flush=True)
# AB_ENV_A="K=V,...": environment for creating plan A only (plan-time switches)
env_a = dict(kv.split("=", 1) for kv in os.environ.get("AB_ENV_A", "").split(",") if kv)
old_env = {k: os.environ.get(k) for k in env_a}
os.environ.update(env_a)
plan_a = esa.plan(minlen, begin, end)
for k, v in old_env.items():
    if v is None:
        os.environ.pop(k, None)
    else:
        os.environ[k] = v
G._lib = LB
plan_b = esa.plan(minlen, begin, end)
G._lib = LA
s = torch.cuda.current_stream()
sp = s.cuda_stream


def timed(L, p, n=30):
    """The step in ms, from a pass without K1 events (an event record between
    K1 and K1b costs ~5.7 us, profiles/r04r/); K1 from the plan's events
    around every K1 of a pass before it."""
    import ctypes
    for _ in range(3):
        L.gt_smax_plan_run(p.plan, sp)
    L.gt_smax_plan_timing(p.plan, n)           # K1 events of this pass
    for _ in range(n):
        L.gt_smax_plan_run(p.plan, sp)
    torch.cuda.synchronize()
    ms, k = ctypes.c_double(), ctypes.c_int()
    L.gt_smax_plan_timing_read(p.plan, ctypes.byref(ms), ctypes.byref(k))
    k1.setdefault(id(L), []).append(ms.value / max(k.value, 1))
    L.gt_smax_plan_timing(p.plan, 0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(n):
        L.gt_smax_plan_run(p.plan, sp)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


k1 = {}


ta, tb = [], []
for r in range(rounds):
    if r % 2 == 0:                    # alternate which build goes first
        a = timed(LA, plan_a)
        b = timed(LB, plan_b)
    else:
        b = timed(LB, plan_b)
        a = timed(LA, plan_a)
    ta.append(a)
    tb.append(b)
    print("round %d: A %.4f ms  B %.4f ms  B/A %.3f" % (r, a, b, b / a), flush=True)
ta.sort()
tb.sort()
print("median step: A %.4f ms, B %.4f ms, B/A %.4f" % (ta[len(ta) // 2], tb[len(tb) // 2],
                                                        tb[len(tb) // 2] / ta[len(ta) // 2]))
ka, kb = sorted(k1[id(LA)]), sorted(k1[id(LB)])
print("median K1: A %.4f ms, B %.4f ms; rest of the step: A %.4f ms, B %.4f ms"
      % (ka[len(ka) // 2], kb[len(kb) // 2], ta[len(ta) // 2] - ka[len(ka) // 2],
         tb[len(tb) // 2] - kb[len(kb) // 2]))

# both plans' last outputs must agree record for record
na = plan_a.fetch_count()
ra = plan_a.fetch_triples()
G._lib = LB
nb = plan_b.fetch_count()
rb = plan_b.fetch_triples()
G._lib = LA
same = na == nb and bool((ra == rb).all())
print("outputs A == B: %s (%d / %d records)" % (same, na, nb), flush=True)
G._lib = LB
plan_b.close()
G._lib = LA
plan_a.close()

#!/usr/bin/env python3
"""GPU scenario of tests/test_runtime_gpu.py::test_f2_f3_plans_do_not_wait_for_other_streams,
run in a fresh process (three streams on distinct hardware queues).  Prints
one JSON line: the F2/F3 calls that returned only after the busy stream
finished ("waited", empty when the calls are stream-ordered), timings and
the parity checks."""
import ctypes
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

import genometools_smax_amd as G  # noqa: E402
import oracle_lib as O  # noqa: E402
import torch  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                               ctypes.c_void_p]
big = G.DeviceEsa(G.synth_genome("uniform", 100_000_000, 7, threads=8), device=0)
small_text = G.synth_genome("uniform", 2_000_000, 3, threads=8)
small = G.DeviceEsa(small_text, device=0, keep_suftab=True)
host = small.download(suftab=True)
N = small.nonspecials
sa, sb, sc = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
# every buffer the F2/F3 calls take, allocated (and cached) beforehand:
# a first hipMalloc may wait for the device
for _ in range(2):
    q = small.lcpitv_plan(stream=sb.cuda_stream)
    q.events(torch.empty(7 * q.num_events(), dtype=torch.int64, device="cuda").data_ptr(),
             sb.cuda_stream)
    q.close()
    q = small.maxpairs_plan(14, stream=sc.cuda_stream)
    q.count(sc.cuda_stream)
    q.total()
    q.close()
ev = torch.empty(7 * (N + 2 * N), dtype=torch.int64, device="cuda")
itv = torch.empty(5 * N, dtype=torch.int64, device="cuda")
plan = big.plan(20)
plan.run(sa.cuda_stream)
torch.cuda.synchronize()
done = ctypes.c_void_p()
assert hip.hipEventCreate(ctypes.byref(done)) == 0
# stream a: smax passes around a spin kernel of ~1 s (the passes alone
# finish faster on the device than the host can enqueue them)
with torch.cuda.stream(sa):
    for _ in range(10):
        plan.run(sa.cuda_stream)
    torch.cuda._sleep(2_000_000_000)
    for _ in range(10):
        plan.run(sa.cuda_stream)
assert hip.hipEventRecord(done, ctypes.c_void_p(sa.cuda_stream)) == 0
waited = []

def check(what):
    if hip.hipEventQuery(done) != 600:          # 600 = hipErrorNotReady
        waited.append((what, round(time.perf_counter() - t1, 4)))

t1 = time.perf_counter()
f3 = small.lcpitv_plan(stream=sb.cuda_stream)
check("lcpitv plan create")
nev = f3.num_events()
f3.events(ev.data_ptr(), sb.cuda_stream)
n_itv, itv_ptr = f3.intervals()
assert hip.hipMemcpyAsync(itv.data_ptr(), itv_ptr, 40 * n_itv, 3, sb.cuda_stream) == 0
check("lcpitv events")
f2 = small.maxpairs_plan(14, stream=sc.cuda_stream)
check("maxpairs plan create")
f2.count(sc.cuda_stream)
total = f2.total()
check("maxpairs count + total")
sb.synchronize()
check("stream b")
f3.close()
f2.close()
check("plan deletes")
t_calls = time.perf_counter() - t1
torch.cuda.synchronize()
t_all = time.perf_counter() - t1
got = itv[: 5 * n_itv].cpu().numpy().view(np.uint64).reshape(-1, 5)
res = {"waited": waited, "t_calls": t_calls, "t_all": t_all,
       "intervals_equal": bool(np.array_equal(got, O.lcp_intervals(host["lcptab"], host["llvtab"], N,
                                                                   N))),
       "events_count_ok": nev == N + 2 * n_itv}
lcp = host["lcptab"].astype(np.uint64)
if len(host["llvtab"]):
    lcp[host["llvtab"][:, 0].astype(np.int64)] = host["llvtab"][:, 1]

class _E:
    pass
e = _E()
e.lcp, e.suftab, e.nonspecials = lcp, host["suftab"].astype(np.uint64), N
e.text = small_text
res["pairs_equal"] = bool(total == len(O.maxpairs(e, 14)) and total > 100)
res["pairs"] = total
hip.hipEventDestroy(done)
plan.close()
big.release()
small.release()
print(json.dumps(res), flush=True)

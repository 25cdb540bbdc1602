#!/usr/bin/env python3
"""Diagnostic: K1 time over the 64-bit builder's tables as built, and over
fresh copies of the same tables (new allocations made after the build's
temporaries are gone), to see whether table placement costs K1 time.
Args: kind bases minlen"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import genometools_smax_amd as G  # noqa: E402
import torch  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "plant"
bases = int(float(sys.argv[2])) if len(sys.argv) > 2 else 3_000_000_000
minlen = int(sys.argv[3]) if len(sys.argv) > 3 else 50


def view(ptr, nbytes):
    class _V:
        __cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                    "version": 2}
    return torch.as_tensor(_V(), device="cuda")


def k1(lcp, pk, esa, local):
    p = G.SmaxPlan(lcp, None, esa.esa.llvtab_dev, esa.numllv, 0, local, 1, esa.nonspecials,
                   esa.nonspecials, minlen, 0, 0, bwtpk_ptr=pk)
    p.run()
    torch.cuda.synchronize()
    p.enable_timing(10)
    for _ in range(10):
        p.run()
    ms, k = p.kernel_ms()
    cnt = p.fetch_count()
    p.close()
    return ms / k, cnt


text = G.synth_genome(kind, bases, 1)
esa = G.DeviceEsa64(text)
del text
if len(sys.argv) > 4:                  # idle before measuring (clock state)
    import time
    time.sleep(float(sys.argv[4]))
local = esa.row_hi - esa.row_lo
pkb = 8 * G.pk_groups(local)
t0, c0 = k1(esa.esa.lcptab_dev, esa.esa.bwtpk_dev, esa, local)
print("as built:   K1 %.3f ms (%d intervals)  lcp %#x pk %#x" % (t0, c0, esa.esa.lcptab_dev,
                                                                    esa.esa.bwtpk_dev), flush=True)
lcp2 = G.DeviceTable(0, local)
pk2 = torch.empty(pkb, dtype=torch.uint8, device="cuda")
view(lcp2.ptr, local).copy_(view(esa.esa.lcptab_dev, local))
pk2.copy_(view(esa.esa.bwtpk_dev, pkb))
torch.cuda.synchronize()
t1, c1 = k1(lcp2.ptr, pk2.data_ptr(), esa, local)
print("fresh copy: K1 %.3f ms (%d intervals)  lcp %#x pk %#x" % (t1, c1, lcp2.ptr, pk2.data_ptr()),
      flush=True)
t2, c2 = k1(esa.esa.lcptab_dev, esa.esa.bwtpk_dev, esa, local)
print("as built:   K1 %.3f ms (%d intervals)" % (t2, c2), flush=True)
# warm-up trend: batches of 10 runs right after each other
p = G.SmaxPlan(esa.esa.lcptab_dev, None, esa.esa.llvtab_dev, esa.numllv, 0, local, 1,
               esa.nonspecials, esa.nonspecials, minlen, 0, 0, bwtpk_ptr=esa.esa.bwtpk_dev)
trend = []
for b in range(12):
    p.enable_timing(10)
    for _ in range(10):
        p.run()
    ms, k = p.kernel_ms()
    trend.append(ms / k)
print("trend (ms per K1, batches of 10):", " ".join("%.3f" % x for x in trend), flush=True)
p.close()

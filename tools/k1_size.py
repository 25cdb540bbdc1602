#!/usr/bin/env python3
"""Diagnostic: K1 time per suffix row vs genome size (64-bit builder
tables), to separate size effects (address translation, table placement)
from per-row work.  Args: kind minlen size1,size2,..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import genometools_smax_amd as G  # noqa: E402
import torch  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "plant"
minlen = int(sys.argv[2]) if len(sys.argv) > 2 else 50
sizes = [int(float(x)) for x in (sys.argv[3] if len(sys.argv) > 3 else "3e9,6e9,12e9").split(",")]
dbgs = [int(x, 0) for x in (sys.argv[4] if len(sys.argv) > 4 else "0").split(",")]
for n in sizes:
    text = G.synth_genome(kind, n, 1)
    esa = G.DeviceEsa64(text)
    del text
    for dbg in dbgs:
        os.environ["GT_SMAX_DEBUG"] = str(dbg)
        p = esa.plan(minlen)
        p.run()
        torch.cuda.synchronize()
        p.enable_timing(10)
        for _ in range(10):
            p.run()
        ms, k = p.kernel_ms()
        k1 = ms / k
        print("%s %.1e dbg %d rows=%d llv=%d K1 %.3f ms = %.1f ps/row, deferred %d of %d tiles"
              % (kind, n, dbg, esa.nonspecials, esa.numllv, k1, k1 * 1e9 / esa.nonspecials,
                 p.deferred_tiles(), p.num_tiles), flush=True)
        p.close()
    os.environ["GT_SMAX_DEBUG"] = "0"
    esa.release()
    torch.cuda.synchronize()

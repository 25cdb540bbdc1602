#!/usr/bin/env python3
"""Diagnostic: K1b cost per tile (GT_SMAX_DEBUG=32768: each K1b tile stores its
wave's cycle count / 16 instead of its record count; K1 tiles keep counts
<= 64).  Optional extra bits: 65536 stamps after the window load, 131072
after the ballots, 262144 after the evaluation (workgroup kernel).
Args: kind bases minlen [extra_dbg] [shard/of, e.g. 0/8]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import genometools_smax_amd as G  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "human"
bases = int(float(sys.argv[2])) if len(sys.argv) > 2 else 3_000_000_000
minlen = int(sys.argv[3]) if len(sys.argv) > 3 else 20
extra = int(sys.argv[4]) if len(sys.argv) > 4 else 0
shard = sys.argv[5] if len(sys.argv) > 5 else "0/1"
si, sw = (int(x) for x in shard.split("/"))
text = G.synth_genome(kind, bases, {"uniform": 42, "human": 1, "plant": 2}[kind])
esa = G.DeviceEsa(text)
del text
N = esa.nonspecials
begin, end = 1 + (N - 1) * si // sw, 1 + (N - 1) * (si + 1) // sw
print("shard %d/%d rows [%d, %d)" % (si, sw, begin, end), flush=True)
for label, dbg in (("whole tile", 32768), ("window load", 32768 | 65536),
                   ("load+ballots", 32768 | 131072), ("+evaluation", 32768 | 262144),
                   ("loads landed", 32768 | 524288), ("+LDS writes", 32768 | 1048576)):
    os.environ["GT_SMAX_DEBUG"] = str(dbg | extra)
    p = esa.plan(minlen, begin, end)
    p.run()
    torch.cuda.synchronize()
    counts, deferred = p.debug_tiles()
    c = counts.astype(np.int64)
    k1b = c[c > 64] * 16
    print("%-13s K1b tiles (cycles > 1024): %d; cycles p50 %d p90 %d max %d; sum %.3g"
          % (label, len(k1b), np.median(k1b) if len(k1b) else 0,
             np.percentile(k1b, 90) if len(k1b) else 0, k1b.max() if len(k1b) else 0, k1b.sum()),
          flush=True)
    top = np.argsort(c)[-5:][::-1]
    print("   slowest tiles:", ", ".join("%d:%d" % (t, c[t] * 16) for t in top), flush=True)
    p.close()

#!/usr/bin/env python3
"""Diagnostic A/B: C3 step and K1 times of the library named by GT_SMAX_LIB
(default: the in-tree build); one ESA build, 5 x 30 timed steps."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import genometools_smax_amd as G  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "human"
bases = int(float(sys.argv[2])) if len(sys.argv) > 2 else 3_000_000_000
minlen = int(sys.argv[3]) if len(sys.argv) > 3 else 20
text = G.synth_genome(kind, bases, {"uniform": 42, "human": 1, "plant": 2}[kind])
esa = G.DeviceEsa(text) if len(text) + 1 < 2 ** 32 else G.DeviceEsa64(text)
del text
s = torch.cuda.current_stream().cuda_stream
p = esa.plan(minlen)
for _ in range(3):
    p.run(s)
steps, k1s = [], []
for rep in range(5):
    p.enable_timing(30)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(30):
        p.run(s)
    torch.cuda.synchronize()
    steps.append((time.perf_counter() - t0) / 30 * 1e3)
    k1, n = p.kernel_ms()
    k1s.append(k1 / max(n, 1))
print("%s: step min %.3f med %.3f ms, K1 min %.3f med %.3f ms, %d intervals"
      % (os.environ.get("GT_SMAX_LIB", "in-tree"), min(steps), sorted(steps)[2], min(k1s),
         sorted(k1s)[2], p.fetch_count()), flush=True)

#!/usr/bin/env python3
"""Diagnostic: C3 step time (K0, K1, static K1b, runtime K1b, K3) for each
placement of the static K1b list (GT_SMAX_K1B_MODE 0..4, see
gt_smax_plan_create), K1 time by HIP events, one ESA build."""
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
esa = G.DeviceEsa(text)
del text
s = torch.cuda.current_stream().cuda_stream
ref = None
for rep in range(2):
    for mode in (0, 2, 4):
        os.environ["GT_SMAX_K1B_MODE"] = str(mode)
        p = esa.plan(minlen)
        for _ in range(3):
            p.run(s)
        p.enable_timing(30)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(30):
            p.run(s)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 30 * 1e3
        k1, n = p.kernel_ms()
        c = p.fetch_count()
        if ref is None:
            ref = c
        print("mode %d: step %.3f ms, K1 %.3f ms, %d intervals%s"
              % (mode, dt, k1 / max(n, 1), c, "" if c == ref else " MISMATCH"), flush=True)
        p.close()

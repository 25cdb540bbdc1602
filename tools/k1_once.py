#!/usr/bin/env python3
"""Diagnostic / profiling driver: build one BASELINE config's ESA exactly as
bench.py does (same generator, seed, builder and minlen) and run the smax
pass a few times, for rocprofv3 counter passes on the scan kernels.

  k1_once.py CONFIG [RUNS]          CONFIG = bench.py config (c2, c3, c5 ...)
  k1_once.py KIND BASES [RUNS]      older form: KIND genome of BASES, minlen 20
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import genometools_smax_amd as G  # noqa: E402
import torch  # noqa: E402

if sys.argv[1] in bench.CONFIGS:
    cfg = bench.CONFIGS[sys.argv[1]]
    kind, bases, seed, minlen = cfg["kind"], cfg["bases"], cfg["seed"], cfg["minlen"]
    runs = int(sys.argv[2]) if len(sys.argv) > 2 else 3
else:
    kind = sys.argv[1]
    bases = int(float(sys.argv[2])) if len(sys.argv) > 2 else 300_000_000
    runs = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    seed, minlen = (1 if kind != "uniform" else 42), 20
text = G.synth_genome(kind, bases, seed, threads=16)
if len(text) + 1 >= 2 ** 32:
    esa = G.DeviceEsa64(text, device=0)
else:
    esa = G.DeviceEsa(text, device=0)
del text
p = esa.plan(minlen)
for _ in range(runs):
    p.run()
torch.cuda.synchronize()
print("intervals", p.fetch_count(), "build", G.build_id(), flush=True)
p.close()
esa.release()

#!/usr/bin/env python3
"""Diagnostic: build one synthetic ESA and run the smax pass a few times
(for rocprofv3 counter collection on K1)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import genometools_smax_amd as G
import torch

kind = sys.argv[1] if len(sys.argv) > 1 else "human"
bases = int(float(sys.argv[2])) if len(sys.argv) > 2 else 300_000_000
runs = int(sys.argv[3]) if len(sys.argv) > 3 else 3
text = G.synth_genome(kind, bases, 1 if kind != "uniform" else 42)
esa = G.DeviceEsa(text)
p = esa.plan(20)
for _ in range(runs):
    p.run()
torch.cuda.synchronize()
print("intervals", p.fetch_count(), flush=True)

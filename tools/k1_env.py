#!/usr/bin/env python3
"""Diagnostic: K1 time under environment variants, one process, interleaved
rounds.  Variants: 'A=1,B=2|A=3|' ('' = no extra variables).  Outputs under
ablation bits are wrong -- timing only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import genometools_smax_amd as G
import torch

kind = sys.argv[1] if len(sys.argv) > 1 else "human"
bases = int(float(sys.argv[2])) if len(sys.argv) > 2 else 300_000_000
variants = sys.argv[3].split("|") if len(sys.argv) > 3 else [""]
text = G.synth_genome(kind, bases, 1 if kind != "uniform" else 42)
esa = G.DeviceEsa(text)
res = {v: [] for v in variants}
base_env = dict(os.environ)
for rnd in range(int(os.environ.get("ROUNDS", "3"))):
    for v in variants:
        os.environ.clear()
        os.environ.update(base_env)
        for kv in filter(None, v.split(",")):
            k, x = kv.split("=")
            os.environ[k] = x
        p = esa.plan(20)
        p.run(); torch.cuda.synchronize()
        p.enable_timing(10)
        for _ in range(10):
            p.run()
        ms, n = p.kernel_ms()
        res[v].append(ms / n)
        p.close()
for v in variants:
    print("%-40s K1 ms: min %.4f med %.4f" % (v or "(default)", min(res[v]), sorted(res[v])[len(res[v]) // 2]), flush=True)

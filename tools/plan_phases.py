#!/usr/bin/env python3
"""Plan-creation cost on a bench config: builds the config's ESA on the GPU,
then creates (and deletes) the smax plan REPEAT times, printing the wall
time of each create and, with GT_SMAX_TIMING=1 in the environment, the
library's per-phase marks (stderr).

  GT_SMAX_TIMING=1 python tools/plan_phases.py [c3] [--repeat 3]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", nargs="?", default="c3")
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--bases", type=float, default=None)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    import genometools_smax_amd as G
    cfg = dict(bench.CONFIGS[a.config])
    if a.bases:
        cfg["bases"] = int(a.bases)
    text = G.synth_genome(cfg["kind"], cfg["bases"], cfg["seed"], threads=16)
    N = len(text) - int(np.count_nonzero(text >= 254))
    n = len(text)
    if n + 1 >= 2 ** 32:   # as bench.py: the 64-bit range builder over all rows
        esa = G.DeviceEsa64(text, device=0, row_lo=0, row_hi=n + 1)
        del text
    else:
        esa = G.DeviceEsa(text, device=0, keep_suftab=False)
    torch.cuda.synchronize()
    for r in range(a.repeat):
        print("[plan %d]" % r, file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        plan = esa.plan(cfg["minlen"], 1, N, packed=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        plan.run(torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        print("plan %d: %.3f ms, %d records" % (r, dt * 1e3, plan.fetch_count()), flush=True)
        plan.close()


if __name__ == "__main__":
    main()

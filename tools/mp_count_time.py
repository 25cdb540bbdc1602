#!/usr/bin/env python3
"""Time gt_maxpairs_plan_count alone on C2's table (bench.py --path maxpairs
input) under runtime settings, one line per setting:

  mp_count_time.py [K=V[,K=V] ...]      each setting in turn, same plan

Settings are read per call (GT_MP_LOOKBACK, GT_MP_RANK_MAX), so one process
and one plan serve all of them; HIP events bracket 200 passes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402
import genometools_smax_amd as G  # noqa: E402

cfg = bench.CONFIGS["c2"]
text = G.synth_genome(cfg["kind"], cfg["bases"], cfg["seed"], threads=16)
esa = G.DeviceEsa(text, device=0, keep_suftab=True)
plan = esa.maxpairs_plan(cfg["minlen"])
s = torch.cuda.current_stream().cuda_stream
for st in sys.argv[1:] or [""]:
    kv = dict(x.split("=", 1) for x in st.split(",") if x)
    saved = {k: os.environ.get(k) for k in kv}
    os.environ.update(kv)
    for _ in range(20):
        plan.count(s)
    total = plan.total()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(200):
        plan.count(s)
    b.record()
    torch.cuda.synchronize()
    print("%-40s count pass %.2f us  total %d" % (st or "default", a.elapsed_time(b) * 5.0, plan.total()),
          flush=True)
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
plan.close()

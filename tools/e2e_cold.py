#!/usr/bin/env python3
"""Cold end-to-end of the drop-in entry point (bench.py's "cold" leg alone):
build a config's ESA on the GPU, download the host tables, then time the
first (and second) gt_smax_hip_enumerate_to_buffer call of a FRESH process
(bin/gt-smax-e2e), with the GT_SMAX_TIMING phases of its first call.

  e2e_cold.py CONFIG [CALLS] [K=V[,K=V] ...]
      CONFIG = bench.py config (c2, c3, c5 ...); each K=V,... setting is a
      further fresh process under those environment variables (runtime
      switches such as GT_SMAX_RING, GT_SMAX_STAGE_MB), all on the same tables
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
import genometools_smax_amd as G  # noqa: E402

cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 3
text = G.synth_genome(cfg["kind"], cfg["bases"], cfg["seed"], threads=16)
esa = G.DeviceEsa(text, device=0) if len(text) + 1 < 2 ** 32 else G.DeviceEsa64(text, device=0)
del text
host = esa.download()
n, N = esa.totallength, esa.nonspecials
esa.release()
G.release_cache()
import oracle_lib  # noqa: E402  (the checker)
want = oracle_lib.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], N, cfg["minlen"], threads=16)
settings = sys.argv[3:] or [""]
out = {}
for i, st in enumerate(settings):
    kv = dict(x.split("=", 1) for x in st.split(",") if x)
    saved = {k: os.environ.get(k) for k in kv}
    os.environ.update(kv)
    try:
        out["%d:%s" % (i, st or "default")] = bench.cold_e2e(G, host, n, N, cfg["minlen"], want, bench.log, calls=calls)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
if len(settings) == 1:
    print(json.dumps(out["0:" + (settings[0] or "default")], indent=1))
else:
    print(json.dumps(out, indent=1))
    for k, r in out.items():
        if not r or "seconds" not in r:
            print("%-34s failed" % k, file=sys.stderr)
            continue
        h2d = lambda ph: " ".join(x for x in (ph or []) if x.split()[0].startswith("h2d")) or "-"
        print("%-34s first %.4f s  second %s s  h2d %s / %s" %
              (k, r["seconds"], r["second_call_s"], h2d(r["phases_first_call"]),
               h2d(r.get("phases_second_call"))), file=sys.stderr)

#!/usr/bin/env python3
"""Cold end-to-end of the drop-in entry point (bench.py's "cold" leg alone):
build a config's ESA on the GPU, download the host tables, then time the
first (and second) gt_smax_hip_enumerate_to_buffer call of a FRESH process
(bin/gt-smax-e2e), with the GT_SMAX_TIMING phases of its first call.

  e2e_cold.py CONFIG [CALLS]       CONFIG = bench.py config (c2, c3, c5 ...)
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
res = bench.cold_e2e(G, host, n, N, cfg["minlen"], want, bench.log, calls=calls)
print(json.dumps(res, indent=1))

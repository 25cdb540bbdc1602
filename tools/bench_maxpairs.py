#!/usr/bin/env python3
"""Secondary bench line: GPU maximal pairs (`gt repfind -l
minlen`) on the C2 workload (100 Mbp uniform ACGT, seed 42, minlen 20),
tables (with the suffix array) resident in HBM.  A step is one count pass +
scan + emission pass.  CPU baseline: the oracle's restatement of the
reference's bottom-up maxpairs traversal (orc_maxpairs, single core) on the
same tables.  Also times the step with the emission in the reference's
order (count + gt_maxpairs_plan_emit_ordered, which synchronises).  Prints
one JSON line."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import genometools_smax_amd as G  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bases", type=int, default=100_000_000)
    ap.add_argument("--kind", default="uniform")
    ap.add_argument("--minlen", type=int, default=20)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    text = G.synth_genome(args.kind, args.bases, 42 if args.kind == "uniform" else 1)
    esa = G.DeviceEsa(text, keep_suftab=True)
    N = esa.nonspecials
    plan = esa.maxpairs_plan(args.minlen)
    plan.count()
    total = plan.total()
    out = torch.empty(max(3 * total, 3), dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream

    def step():
        plan.count(s)
        plan.emit(out.data_ptr(), total, s)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / args.steps
    outo = torch.empty(max(3 * total, 3), dtype=torch.int64, device="cuda")

    def step_ordered():
        plan.count(s)
        plan.emit_ordered(outo.data_ptr(), total, s)

    for _ in range(args.warmup):
        step_ordered()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step_ordered()
    torch.cuda.synchronize()
    elo = (time.perf_counter() - t0) / args.steps
    cpu = None
    if not args.no_cpu_baseline:
        import oracle_lib as O
        h = esa.download(suftab=True)
        lcp = h["lcptab"].astype(np.uint64)
        if len(h["llvtab"]):
            lcp[h["llvtab"][:, 0].astype(np.int64)] = h["llvtab"][:, 1]

        class _E:
            pass
        e = _E()
        e.lcp, e.suftab, e.text, e.nonspecials = lcp, h["suftab"], text, N
        t0 = time.perf_counter()
        ref = O.maxpairs(e, args.minlen)
        tc = time.perf_counter() - t0
        got = out[: 3 * total].cpu().numpy().view(np.uint64).reshape(-1, 3)

        def norm(p):
            q = np.stack([p[:, 0], np.minimum(p[:, 1], p[:, 2]), np.maximum(p[:, 1], p[:, 2])], 1)
            return q[np.lexsort((q[:, 2], q[:, 1], q[:, 0]))]
        same = len(ref) == total and np.array_equal(norm(ref), norm(got))
        goto = outo[: 3 * total].cpu().numpy().view(np.uint64).reshape(-1, 3)
        refo = np.stack([ref[:, 0], np.minimum(ref[:, 1], ref[:, 2]),
                         np.maximum(ref[:, 1], ref[:, 2])], 1) if len(ref) else ref
        same_order = len(ref) == total and np.array_equal(refo, goto)
        cpu = {"value": N / tc, "unit": "suffix-positions/s", "cores": 1, "kind": "port",
               "sample": "oracle orc_maxpairs (restated gt_esa_bottomup_maxpairs, 1 core) over all "
                         "%d rows: %.2fs; pair set identical to the GPU's: %s; reference emission order "
                         "identical to the GPU's ordered pass: %s" % (N, tc, same, same_order)}
    # the host-table entry points (the `gt repfind -l` runner's drop-in,
    # src/match/esa-maxpairs.c:476-520, and the F3 tree): pageable host
    # tables -> staged H2D -> count/emit (reference order) -> D2H, in this
    # process after the device steps; and the F3 lcp-interval tree likewise
    h = esa.download(suftab=True)
    n = esa.totallength
    plan.close()
    host = {}
    for name, fn in (("maxpairs_enumerate_to_buffer",
                      lambda: G.enumerate_maxpairs(h["lcptab"], h["llvtab"], h["bwttab"], h["suftab"],
                                                   n, N, args.minlen)),
                     ("lcpitv_enumerate_to_buffer",
                      lambda: G.enumerate_lcp_intervals(h["lcptab"], h["llvtab"], n, N))):
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            r = fn()
            ts.append(time.perf_counter() - t0)
        host[name] = {"seconds_first": round(ts[0], 4), "seconds_best": round(min(ts), 4),
                      "value_best": N / min(ts), "records": len(r)}
        if name.startswith("maxpairs") and cpu is not None:
            host[name]["identical_to_oracle"] = bool(np.array_equal(r, ref))
        del r
    print(json.dumps({
        "metric": "suffix-positions/s (maximal pairs, gt repfind -l %d)" % args.minlen,
        "value": N / el, "unit": "suffix-positions/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": el * 1e3, "higher_is_better": True,
        "dtype": "u32", "data": "synthetic",
        "config": {"workload": "%d bp synthetic %s DNA, minlen=%d" % (args.bases, args.kind, args.minlen),
                   "nonspecials": N},
        "maximal_pairs": total, "maximal_pairs_per_s": total / el,
        "ms_per_step_reference_order": elo * 1e3,
        "host_entry_points": host,
        "cpu_baseline": cpu}), flush=True)
    esa.release()


if __name__ == "__main__":
    main()

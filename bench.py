#!/usr/bin/env python3
"""bench.py -- throughput of the smax hot path on MI355X (BASELINE.json metric).

One "step" = one smax pass over the whole suffix array of the workload:
the fused plateau-scan / left-diversity / ordered-compaction kernel K1
(plus K1b for deferred tiles and the block sums, K3 compaction) on every rank's suffix-array range and, with
N > 1, the RCCL all-gather of the fixed-size boundary records and the stitch
kernel.  The LCP/BWT/.llv tables are resident in HBM before timing starts
(built on each GPU by the repo's GPU suffixerator replacement from a
deterministic synthetic genome; ESA construction is reported as setup).
Before the warmup steps the device is primed with untimed full passes for
--prime-s seconds (the clocks ramp over ~20 passes after the setup's idle
periods; the count is reported under "priming").

Workload (default, configs[2] of BASELINE.json, where the ≥10x / ≥50 % HBM
target is quoted): 3 Gbp synthetic human-like DNA (40 % interspersed repeats,
STRs, segmental duplications, N gaps, 24 sequences), minlen 20.  --config c2
runs configs[1] (100 Mbp uniform ACGT).  N GPUs shard the same suffix array
by range (strong scaling): value = nonspecials / max-over-ranks step time.

Prints ONE JSON line on rank 0 (contract in the task statement), with
"roofline" for K1 (algorithmic bytes = 2 B per suffix row + 16 B per .llv
entry + 16 B per emitted record, SURVEY.md §8(d), over the average K1 duration from HIP events recorded
on K1's stream around every 8th K1 launch of the timed region) and, at N = 1, "cpu_baseline": the
oracle's single-core linear scan (oracle/smax_oracle.c orc_linsmax, the
repo's CPU esa_linsmax restatement) timed on this host over the same tables.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = ("suffix-positions/s (and supermax repeats/s) at minlen=20; % HBM roofline; "
          "1/2/4/8 GPU")
HBM_PEAK_GBS = 8000.0

CONFIGS = {
    "c3": dict(kind="human", bases=3_000_000_000, seed=1, minlen=20,
               workload="3 Gbp synthetic human-like DNA (40% repeats), minlen=20"),
    # configs[4]: 12 Gbp plant-like (80 % LTR-like families, nested
    # insertions), minlen 50, > 2^32 suffixes: the 64-bit ESA builder
    "c5": dict(kind="plant", bases=12_000_000_000, seed=2, minlen=50,
               workload="12 Gbp synthetic plant-like DNA (80% LTR-like repeats), minlen=50"),
    # C5's profile at 4.2 Gbp (round-1 proxy, kept for comparison)
    "c5p": dict(kind="plant", bases=4_200_000_000, seed=2, minlen=50,
                workload="4.2 Gbp synthetic plant-like DNA (80% LTR-like repeats), minlen=50"),
    "c2": dict(kind="uniform", bases=100_000_000, seed=42, minlen=20,
               workload="100 Mbp synthetic uniform ACGT, minlen=20"),
}


def host_cpu():
    """Host CPU identity for the cpu_baseline object."""
    model = None
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(),
            "affinity_cpus": len(os.sched_getaffinity(0))}


def cgroup_cpus():
    """CPUs the container's cgroup quota allows (cpu.max), None if unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def log(msg):
    print("[bench] " + msg, file=sys.stderr, flush=True)


def cold_e2e(G, host, n, N, minlen, want, log, calls=2, prepared=False):
    """The drop-in entry point's first call in a FRESH process: the host
    tables go to files (untimed), bin/gt-smax-e2e reads them into its own
    memory, initialises the HIP runtime (gt_smax_device_count, timed apart)
    and times `calls` calls of gt_smax_hip_enumerate_to_buffer; the first
    call's triples come back for the parity check.  None when the binary or
    the scratch space is missing.  prepared: the process issues
    gt_smax_hip_prepare at its start, before it reads the tables (as a
    `gt repfind` runner does once the .prj has given the sizes)."""
    import shutil
    import subprocess
    import tempfile
    import numpy as np
    exe = os.path.join(G.BIN_DIR, "gt-smax-e2e")
    if not os.path.exists(exe):
        log("cold end-to-end: %s missing (make -C genometools_smax_amd)" % exe)
        return None
    need = 2 * (n + 1) + host["llvtab"].nbytes + 24 * (len(want) if want is not None else n // 64)
    base = None
    for d in (os.environ.get("GT_SMAX_E2E_DIR"), "/dev/shm", tempfile.gettempdir()):
        try:
            if d and os.path.isdir(d):
                st = os.statvfs(d)
                if st.f_bavail * st.f_frsize > 1.3 * need:
                    base = d
                    break
        except OSError:
            continue
    if base is None:
        log("cold end-to-end: no scratch directory with %.1f GB free" % (need / 1e9))
        return None
    tmp = tempfile.mkdtemp(prefix="gtsmax_e2e_", dir=base)
    try:
        paths = [os.path.join(tmp, x) for x in ("lcp", "bwt", "llv", "out")]
        host["lcptab"].tofile(paths[0])
        host["bwttab"].tofile(paths[1])
        np.ascontiguousarray(host["llvtab"], dtype=np.uint64).tofile(paths[2])
        env = dict(os.environ)
        env["GT_SMAX_TIMING"] = "1"
        if prepared:
            env["GT_SMAX_E2E_PREPARE"] = "1"
        r = subprocess.run([exe, paths[0], paths[1], paths[2], str(n), str(N), str(minlen),
                            str(calls), "1", paths[3]], capture_output=True, text=True,
                           env=env, timeout=600)
        if r.returncode != 0:
            log("cold end-to-end failed (%d): %s" % (r.returncode, r.stderr[-2000:]))
            return {"parity_ok": False, "error": r.stderr[-500:]}
        res = json.loads(r.stdout.strip().splitlines()[-1])
        got = np.fromfile(paths[3], dtype=np.uint64).reshape(-1, 3)
        ok = want is None or bool(np.array_equal(got, want))
        if not ok:
            log("FAIL: cold end-to-end result (%d intervals) differs from the CPU oracle (%d)"
                % (len(got), len(want)))
        phases, phases2, call = [], [], -1
        for ln in r.stderr.splitlines():
            if ln.startswith("[gt_smax call]"):
                call = int(ln.split("]", 1)[1])
            elif ln.startswith("[gt_smax timing]") and call in (0, 1):
                (phases if call == 0 else phases2).append(" ".join(ln.split("]", 1)[1].split()))
        t = res["calls_s"]
        log("cold end-to-end%s: HIP init %.3fs, calls %s s" % (" (prepared)" if prepared else "", res["hip_init_s"], t))
        return {"parity_ok": ok, "value": N / t[0], "unit": "suffix-positions/s",
                "seconds": round(t[0], 4), "hip_init_s": round(res["hip_init_s"], 4),
                "prepared": bool(res.get("prepared")), "table_read_s": round(res.get("read_s", 0.0), 4),
                "second_call_s": round(t[1], 4) if len(t) > 1 else None,
                "process": "fresh process (bin/gt-smax-e2e, C, links libgtsmax_hip.so only): "
                           "first gt_smax_hip_enumerate_to_buffer call; the HIP runtime's "
                           "initialisation (gt_smax_device_count before it) is hip_init_s",
                "phases_first_call": phases or None,
                "phases_second_call": phases2 or None}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main_lcpitv(args):
    """F3 leg: the generic bottom-up traversal -- every
    lcp-interval with its father in pop order and the GtESAVisitor event
    stream in the reference's order (/root/reference/src/match/
    esa-bottomup.c:116-273) -- over tables resident in HBM.  A step is one
    gt_lcpitv_plan_create (the interval tree: exact LCP, per-tile ANSV of
    PL / NSE / e, chain depths, the pops' exclusive scan, the pop-ordered
    interval records) + one gt_lcpitv_plan_events pass into a resident
    buffer + gt_lcpitv_plan_delete.  One GPU (--gpus N: replicas).

    Algorithmic bytes per step (the roofline's "achieved", a fixed model, not
    the kernels' traffic -- that is in profiles/r6/pmc_lcpitv_c2.json): per
    row the LCP byte read, its exact u32 written and read twice (1 + 4 + 2 x
    4 B), per interval its 5-word record written (40 B), per event its
    7-word record (56 B) plus the events pass's LCP u32 and 4-byte suffix
    reads (8 B per row)."""
    import numpy as np
    import torch
    import genometools_smax_amd as G

    cfg = dict(CONFIGS[args.config])
    if args.config not in ("c2",) and not args.bases:
        sys.exit("bench.py --path lcpitv: use --config c2 (or --bases): the event stream is 56 B "
                 "per row and per interval end")
    if args.bases:
        cfg["bases"] = args.bases
        cfg["workload"] = cfg["workload"].replace(
            cfg["workload"].split(" synthetic")[0], "%.3g bp" % args.bases)
    cfg["workload"] = cfg["workload"].split(", minlen")[0]
    world, rank, local = rank_env(args)
    torch.cuda.set_device(0 if args.one_gpu else local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")   # replicas: the barrier only
    t0 = time.time()
    text = G.synth_genome(cfg["kind"], cfg["bases"], cfg["seed"], threads=16)
    t_gen = time.time() - t0
    t0 = time.time()
    esa = G.DeviceEsa(text, device=torch.cuda.current_device(), keep_suftab=True)
    t_esa = time.time() - t0
    n, N = esa.totallength, esa.nonspecials
    plan = esa.lcpitv_plan()
    nitv = plan.intervals()[0]
    n_ev = plan.num_events()
    itv0 = None
    if rank == 0 and not args.no_cpu_baseline:
        nn, ptr = plan.intervals()
        itv0 = torch.empty(5 * max(nn, 1), dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()

        class _View:   # the plan's device records, copied out before it closes

            __cuda_array_interface__ = {"shape": (5 * nn,), "typestr": "<i8", "data": (ptr, False),
                                        "version": 2}
        if nn:
            itv0.copy_(torch.as_tensor(_View(), device="cuda"))
    plan.close()
    ev = torch.empty(7 * max(n_ev, 1), dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream

    def step():
        p = esa.lcpitv_plan()
        p.events(ev.data_ptr(), s)
        p.close()

    def step_tree():
        esa.lcpitv_plan().close()

    def timed(fn):
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / args.steps

    t_pr = time.perf_counter()
    while time.perf_counter() - t_pr < args.prime_s:
        step_tree()
    el = timed(step)
    el_tree = timed(step_tree)
    if dist:
        mx = torch.tensor([el, el_tree], dtype=torch.float64)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        el, el_tree = float(mx[0]), float(mx[1])
    alg_tree = N * 13 + nitv * 40
    alg = alg_tree + n_ev * 56 + N * 8
    parity = None
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib as O  # noqa: E402  (the checker, CPU baseline leg only)
        h = esa.download()
        t0 = time.perf_counter()
        ref = O.lcp_intervals(h["lcptab"], h["llvtab"], N, nitv + 1)
        t_cpu = time.perf_counter() - t0
        got = itv0[: 5 * nitv].cpu().numpy().view(np.uint64).reshape(-1, 5)
        same = len(ref) == nitv and bool(np.array_equal(ref, got))
        parity = {"intervals_identical_pop_order": same,
                  "num_events": n_ev, "num_events_expected": N + 2 * nitv,
                  "events": "record for record against the oracle's gt_esa_bottomup stream on the "
                            "fixtures and random texts (tests/test_lcpitv_gpu.py)"}
        cpu = {"value": N / t_cpu, "unit": "suffix-positions/s", "cores": 1, "kind": "port",
               "sample": "oracle orc_lcp_intervals (the gt_esa_bottomup stack walk restated, "
                         "src/match/esa-bottomup.c:116-273, intervals with their fathers, 1 core) "
                         "over all %d rows: %.2fs" % (N, t_cpu), "seconds": round(t_cpu, 3)}
        cpu.update(host_cpu())
        cpu["cgroup_cpus"] = cgroup_cpus()
        del h, ref, got
        if not same or n_ev != N + 2 * nitv:
            log("FAIL: lcp-intervals differ from the oracle: %s" % parity)
            esa.release()
            sys.exit(1)
    if rank == 0:
        achieved = alg / el / 1e9
        print(json.dumps({
            "metric": "suffix-positions/s (generic bottom-up traversal: lcp-interval tree + visitor "
                      "events)",
            "value": world * N / el, "unit": "suffix-positions/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": el * 1e3,
            "higher_is_better": True, "scaling": "weak" if world > 1 else None,
            "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": cfg["workload"], "totallength": n, "nonspecials": N,
                       "path": "lcpitv (F3)",
                       "parallelism": "replicas x%d" % world if world > 1 else "single GPU"},
            "step": "gt_lcpitv_plan_create + gt_lcpitv_plan_events + gt_lcpitv_plan_delete",
            "lcp_intervals": nitv, "visitor_events": n_ev,
            "ms_per_step_tree_only": el_tree * 1e3,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "algorithmic_bytes_per_step": alg,
                         "algorithmic_bytes_per_step_tree_only": alg_tree,
                         "achieved_tree_only": alg_tree / el_tree / 1e9,
                         "note": "whole-pass bytes over the pass time; per-kernel times: the "
                                 "rocprofv3 kernel stats under profiles/"},
            "parity": parity, "cpu_baseline": cpu,
            "setup_s": {"genome": round(t_gen, 2), "gpu_esa_build": round(t_esa, 2)}}), flush=True)
    esa.release()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def main_maxpairs(args):
    """F2 leg: maximal pairs, `gt repfind -l minlen` -- the
    reference's default repfind path (/root/reference/src/match/esa-maxpairs.c:
    476-513, hot loop esa-bottomup-maxpairs.inc:155-243) -- over tables
    resident in HBM (the GPU suffixerator, suffix array kept).  A step is one
    count pass + one emission pass in the reference's emission order
    (gt_maxpairs_plan_count + gt_maxpairs_plan_emit_ordered: the pairs and
    their order equal the reference's GtProcessmaxpairs calls).  One GPU:
    maximal pairs do not shard by suffix-array range without a cross-shard
    pair exchange (pairs span blocks of any length), so --gpus N runs N
    independent replicas.  C3/C5 are refused: a 40-80 % repeat genome of
    3-12 Gbp has ~1e11+ maximal pairs at minlen 20 (copies of a family pair
    quadratically), TBs of output for the reference as for this path.

    Algorithmic bytes per pass (the roofline's "achieved"): the two candidate
    scans over the LCP bytes (count, then ordered write: 2 B/row), and per
    candidate row (LCP >= minlen) its walk in both passes (exact LCP u32 +
    BWT byte, + the 4-byte suffix in the emission pass: 13 B) and list/count/
    offset entries (8 + 4 + 8 B), plus per pair its triple (24 B) and its
    emission-order sort keys (3-4 x 8 B written, LSD passes: + 2 x 16 B per
    key pass)."""
    import numpy as np
    import torch
    import genometools_smax_amd as G

    if args.config not in ("c2",) and not args.bases:
        sys.exit("bench.py --path maxpairs: config %s has ~1e11+ maximal pairs (quadratic in the "
                 "repeat copies); use --config c2 (or --bases for a uniform genome)" % args.config)
    cfg = dict(CONFIGS[args.config])
    if args.bases:
        cfg["bases"] = args.bases
        cfg["workload"] = cfg["workload"].replace(
            cfg["workload"].split(" synthetic")[0], "%.3g bp" % args.bases)
    if args.minlen:
        cfg["minlen"] = args.minlen
    minlen = cfg["minlen"]
    world, rank, local = rank_env(args)
    torch.cuda.set_device(0 if args.one_gpu else local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")   # replicas: the barrier only
    t0 = time.time()
    text = G.synth_genome(cfg["kind"], cfg["bases"], cfg["seed"], threads=16)
    t_gen = time.time() - t0
    t0 = time.time()
    esa = G.DeviceEsa(text, device=torch.cuda.current_device(), keep_suftab=True)
    t_esa = time.time() - t0
    n, N = esa.totallength, esa.nonspecials
    t0 = time.perf_counter()
    plan = esa.maxpairs_plan(minlen)
    torch.cuda.synchronize()
    t_plan = time.perf_counter() - t0
    plan.count()
    total = plan.total()
    ncand = plan.candidates()
    out = torch.empty(max(3 * total, 3), dtype=torch.int64, device="cuda")
    outr = torch.empty(max(3 * total, 3), dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream

    def step():
        plan.count(s)
        plan.emit_ordered(out.data_ptr(), total, s)

    def step_rows():
        plan.count(s)
        plan.emit(outr.data_ptr(), total, s)

    def timed(fn):
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / args.steps

    # priming (clock ramp), as the smax bench
    t_pr = time.perf_counter()
    while time.perf_counter() - t_pr < args.prime_s:
        step_rows()
        torch.cuda.synchronize()
    el = timed(step)
    el_rows = timed(step_rows)
    if dist:
        mx = torch.tensor([el, el_rows], dtype=torch.float64)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        el, el_rows = float(mx[0]), float(mx[1])
    nkeys = 4 if (N.bit_length() + 32) > 64 else 3
    alg = (2 * N + ncand * (5 + 9 + 8 + 4 + 8) + total * (24 + 8 * nkeys + 2 * 16 * nkeys))
    alg_rows = 2 * N + ncand * (5 + 9 + 8 + 4 + 8) + total * 24
    in_mall = N < (256 << 20)      # the LCP bytes stay in the Infinity Cache across passes
    parity = None
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib as O  # noqa: E402  (the checker, CPU baseline leg only)
        h = esa.download(suftab=True)
        lcp = h["lcptab"].astype(np.uint64)
        if len(h["llvtab"]):
            lcp[h["llvtab"][:, 0].astype(np.int64)] = h["llvtab"][:, 1]

        class _E:
            pass
        e = _E()
        e.lcp, e.suftab, e.text, e.nonspecials = lcp, h["suftab"], text, N
        t0 = time.perf_counter()
        ref = O.maxpairs(e, minlen)
        t_cpu = time.perf_counter() - t0
        got = out[: 3 * total].cpu().numpy().view(np.uint64).reshape(-1, 3)
        gotr = outr[: 3 * total].cpu().numpy().view(np.uint64).reshape(-1, 3)

        def norm(p):
            q = np.stack([p[:, 0], np.minimum(p[:, 1], p[:, 2]), np.maximum(p[:, 1], p[:, 2])], 1)
            return q[np.lexsort((q[:, 2], q[:, 1], q[:, 0]))]
        # the ordered pass: the reference's calls, argument order included
        same_order = len(ref) == total and bool(np.array_equal(ref, got))
        same_set = len(ref) == total and bool(np.array_equal(norm(ref), norm(gotr)))
        parity = {"reference_order_identical": same_order, "row_order_pass_same_pair_set": same_set}
        cpu = {"value": N / t_cpu, "unit": "suffix-positions/s", "cores": 1, "kind": "port",
               "sample": "oracle orc_maxpairs (the gt_esa_bottomup_maxpairs stack walk restated, "
                         "src/match/esa-bottomup-maxpairs.inc:136-264, 1 core) over all %d rows: %.2fs"
                         % (N, t_cpu), "seconds": round(t_cpu, 3)}
        cpu.update(host_cpu())
        cpu["cgroup_cpus"] = cgroup_cpus()
        del lcp, h, ref, got, gotr
        if not (same_order and same_set):
            log("FAIL: maxpairs differ from the oracle: %s" % parity)
            plan.close()
            esa.release()
            sys.exit(1)
    if rank == 0:
        achieved = alg / el / 1e9
        print(json.dumps({
            "metric": "suffix-positions/s (maximal pairs, gt repfind -l %d)" % minlen,
            "value": world * N / el, "unit": "suffix-positions/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": el * 1e3,
            "higher_is_better": True, "scaling": "weak" if world > 1 else None,
            "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": cfg["workload"], "minlen": minlen, "totallength": n,
                       "nonspecials": N, "path": "maxpairs (F2)",
                       "parallelism": "replicas x%d" % world if world > 1 else "single GPU"},
            "step": "count pass + emission in the reference's order (gt_maxpairs_plan_count + "
                    "gt_maxpairs_plan_emit_ordered)",
            "maximal_pairs": total, "maximal_pairs_per_s": total / el, "candidate_rows": ncand,
            "ms_per_step_row_order": el_rows * 1e3,
            "roofline": {"bound": "mall" if in_mall else "hbm", "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": None if in_mall else achieved / HBM_PEAK_GBS,
                         "algorithmic_bytes_per_step": alg,
                         "algorithmic_bytes_per_step_row_order": alg_rows,
                         "achieved_row_order": alg_rows / el_rows / 1e9,
                         "note": "whole-pass bytes over the pass time; per-kernel times: the "
                                 "rocprofv3 kernel stats under profiles/"},
            "parity": parity, "cpu_baseline": cpu,
            "setup_s": {"genome": round(t_gen, 2), "gpu_esa_build": round(t_esa, 2),
                        "plan": round(t_plan, 3)}}), flush=True)
    plan.close()
    esa.release()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def launch_ranks(n):
    """`bench.py --gpus N` started as a plain process (no WORLD_SIZE): start
    the N ranks here, one child process per GPU, before anything in this
    process touches HIP or torch.cuda (the parent never imports torch).  Each
    child re-runs this script with RANK / LOCAL_RANK / WORLD_SIZE /
    LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, exactly what
    `python -m torch.distributed.run --nproc-per-node N` hands its workers,
    and inherits stdout/stderr (rank 0 prints the one JSON line).  Returns
    the first non-zero child exit code (the surviving ranks are terminated),
    else 0."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    log("launching %d ranks (127.0.0.1:%d)" % (n, port))
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                log("rank %d exited with %d; stopping the other ranks" % (procs.index(p), code))
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    for p in procs:
        p.wait()
    return rc


def rank_env(args):
    """(world, rank, local) from the launcher's environment; --gpus must
    agree with a set WORLD_SIZE (a mismatch is an error, not a note: the
    line's n_gpus would otherwise not be the count asked for)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" in os.environ and world != args.gpus:
        log("error: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world))
        sys.exit(2)
    return world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--prime-s", type=float, default=0.2,
                    help="untimed device priming before the warmup steps: passes for this many "
                         "seconds (clock ramp after the setup's idle periods)")
    ap.add_argument("--config", default=None, choices=sorted(CONFIGS),
                    help="workload (default: c3 for --path smax, c2 for --path maxpairs)")
    ap.add_argument("--path", default="smax", choices=["smax", "maxpairs", "lcpitv"],
                    help="smax: the hot path (BASELINE metric); maxpairs: the F2 leg, "
                         "`gt repfind -l minlen` maximal pairs in the reference's emission order; "
                         "lcpitv: the F3 leg, the generic bottom-up traversal (intervals + events)")
    ap.add_argument("--bases", type=lambda x: int(float(x)), default=None, help="override genome size")
    ap.add_argument("--minlen", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-end-to-end", action="store_true",
                    help="skip the host-tables (PCIe-inclusive) leg")
    ap.add_argument("--cpu-sample", type=int, default=4_300_000_000,
                    help="max suffix rows timed on the CPU (single-core linear scan)")
    ap.add_argument("--cpu-sample-bottomup", type=int, default=1_000_000_000,
                    help="max suffix rows of the single-core reference-algorithm anchor "
                         "(the bottom-up stack walk, about 20 s per 10^9 rows)")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="threads for the all-core CPU figure (the GPU box's CPU share is 16)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: stage the boundary records through host memory (multi-rank "
                         "rehearsal on one GPU; the measured configuration is nccl = RCCL)")
    ap.add_argument("--one-gpu", action="store_true",
                    help="all ranks on cuda:0 (rehearsal only)")
    ap.add_argument("--esa64", action="store_true",
                    help="build with the 64-bit range builder even when the 32-bit one applies")
    ap.add_argument("--no-parity", action="store_true",
                    help="N > 1: skip gathering every rank's records to rank 0 for the "
                         "whole-table oracle check")
    ap.add_argument("--byte-bwt", action="store_true",
                    help="plan from the byte BWT (plan-time packing) instead of the builder's "
                         "packed BWT")
    ap.add_argument("--launch-probe", default=None, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world, rank, _ = rank_env(args)
    if args.launch_probe:
        # launcher check (tests/test_bench_launch_cpu.py): what this rank was
        # handed, before any GPU or torch import
        print(json.dumps({k: os.environ.get(k) for k in
                          ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                           "MASTER_PORT")}), flush=True)
        sys.exit(3 if args.launch_probe == "fail%d" % rank else 0)
    if args.config is None:
        args.config = "c2" if args.path in ("maxpairs", "lcpitv") else "c3"
    if args.path == "maxpairs":
        return main_maxpairs(args)
    if args.path == "lcpitv":
        return main_lcpitv(args)

    import numpy as np
    import torch
    import genometools_smax_amd as G

    cfg = dict(CONFIGS[args.config])
    if args.bases:
        cfg["bases"] = args.bases
        cfg["workload"] = cfg["workload"].replace(
            cfg["workload"].split(" synthetic")[0], "%.3g bp" % args.bases)
    if args.minlen:
        cfg["minlen"] = args.minlen
    minlen = cfg["minlen"]

    world, rank, local = rank_env(args)
    if args.one_gpu:
        local = 0
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    # ---- setup (untimed): synthetic genome -> GPU ESA.  One GPU and
    # n+1 < 2^32: the 32-bit builder over the whole text; otherwise the
    # 64-bit builder, each rank building only the rows of its suffix-array
    # range (LCP[begin-1 .. end])
    t0 = time.time()
    text = G.synth_genome(cfg["kind"], cfg["bases"], cfg["seed"], threads=16)
    t_gen = time.time() - t0
    log("rank %d: generated %d symbols in %.1fs" % (rank, len(text), t_gen))
    n = len(text)
    N = n - int(np.count_nonzero(text >= 254))
    begin = 1 + (N - 1) * rank // world
    end = 1 + (N - 1) * (rank + 1) // world
    use64 = world > 1 or n + 1 >= 2 ** 32 or args.esa64
    t0 = time.time()
    if use64:
        # one GPU: all n+1 rows (the host-table leg hands the whole tables
        # to the drop-in entry point); ranks: LCP[begin-1 .. end] only
        lo, hi = (0, n + 1) if world == 1 else (begin - 1, end + 1)
        # ranks sharing one GPU (rehearsal) size their sort batches down: each
        # builder would otherwise take what the free HBM allows (~96 B per
        # suffix of a batch) and eight of them at once overcommit the device
        esa = G.DeviceEsa64(text, device=local, row_lo=lo, row_hi=hi,
                            batch_max=(1 << 27) if args.one_gpu and world > 1 else 0)
        builder = "64-bit range builder, rows [%d, %d)" % (lo, hi)
    else:
        esa = G.DeviceEsa(text, device=local, keep_suftab=False)
        builder = "32-bit builder, whole text"
    t_esa = time.time() - t0
    assert (esa.totallength, esa.nonspecials) == (n, N)
    numllv = int(esa.numllv)
    log("rank %d: GPU ESA (%s) n=%d N=%d llv=%d rounds=%d in %.1fs"
        % (rank, builder, n, N, esa.numllv, esa.esa.sort_rounds, t_esa))
    if world > 1 or use64:
        del text
    # the builder emits the packed bit-plane BWT the scan streams (0.5 B/row),
    # so creating the plan reads no BWT bytes: .llv index (u16 values, per-tile
    # windows), the static K1b list and the plan's buffers (--byte-bwt: the
    # plan packs the byte BWT itself, a plan-time pass over 1 B/row)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    plan = esa.plan(minlen, begin, end, packed=not args.byte_bwt)
    torch.cuda.synchronize()
    t_plan = time.perf_counter() - t0
    # a second plan over the same tables (its buffers from the library's
    # allocator cache, the code object loaded): what a caller that keeps the
    # process pays per plan; the first one above includes cold hipMallocs
    t0 = time.perf_counter()
    plan2 = esa.plan(minlen, begin, end, packed=not args.byte_bwt)
    torch.cuda.synchronize()
    t_plan_warm = time.perf_counter() - t0
    plan2.close()
    del plan2
    stream = torch.cuda.current_stream()
    sptr = stream.cuda_stream
    send = recv = None
    staged = world > 1 and args.dist_backend == "gloo"
    if world > 1:
        send = torch.zeros(G.BOUNDARY_BYTES, dtype=torch.uint8, device="cuda")
        recv = torch.zeros(G.BOUNDARY_BYTES * world, dtype=torch.uint8, device="cuda")
        if staged:
            hsend = torch.zeros(G.BOUNDARY_BYTES, dtype=torch.uint8)
            hrecv = torch.zeros(G.BOUNDARY_BYTES * world, dtype=torch.uint8)

    def step():
        if world == 1:
            plan.run(sptr)
            return
        # the one exchange step: all-gather of the fixed-size boundary
        # records, then the stitch kernel resolves spanning plateaus.  The
        # boundary record is final after the scan (part 0), so the all-gather
        # runs on RCCL's stream beside the compaction (part 1); the stitch
        # waits for both.  The send buffer is the plan's own boundary record
        # (zero-copy tensor), so no copy launch sits between scan and collective
        plan.run_part(0, sptr)
        src = bsend[0]
        if src is None:
            plan.copy_boundary(send.data_ptr(), sptr)
            src = send
        if staged:
            hsend.copy_(src)
            work = dist.all_gather_into_tensor(hrecv, hsend, async_op=True)
            plan.run_part(1, sptr)
            work.wait()
            recv.copy_(hrecv)
        else:
            work = dist.all_gather_into_tensor(recv, src, async_op=True)
            plan.run_part(1, sptr)
            work.wait()
        plan.stitch(recv.data_ptr(), world, rank, sptr)

    def boundary_send():
        # the plan's boundary record as the all-gather's send tensor; None:
        # this torch cannot wrap device memory (then copy_boundary each step)
        try:
            return plan.boundary_tensor()
        except Exception as e:  # noqa: BLE001
            log("rank %d: zero-copy boundary send unavailable (%s); copying per step" % (rank, e))
            return None

    bsend = [boundary_send() if world > 1 else None]
    # first pass sizes the output exactly (re-plan on overflow)
    step()
    torch.cuda.synchronize()
    cnt = plan.fetch_count()
    if cnt > plan.capacity:
        log("rank %d: %d intervals > capacity %d, re-planning" % (rank, cnt, plan.capacity))
        plan.close()
        plan = esa.plan(minlen, begin, end, capacity=cnt + 16, packed=not args.byte_bwt)
        bsend[0] = boundary_send() if world > 1 else None

    # device priming (setup, untimed): passes until the device has run them
    # for PRIME_S seconds.  After any idle period -- here the host-side part
    # of the ESA build and plan creation -- the first ~20 passes run up to
    # 30 % slow while the clocks ramp (per-pass times after the build and
    # after a 2 s pause: profiles/r03zh/timing_modes.txt); the driver's 5
    # warmup steps sit inside that ramp.  Every pass is a full pass over the
    # tables (nothing is cached between passes); the count is reported.
    torch.cuda.synchronize()
    t_pr = time.perf_counter()
    n_prime = 0
    while time.perf_counter() - t_pr < args.prime_s:
        for _ in range(8):
            plan.run(sptr)   # local passes only: ranks may run different counts
        torch.cuda.synchronize()
        n_prime += 8
    t_prime = time.perf_counter() - t_pr
    for _ in range(args.warmup):
        step()
    # K1's duration by HIP events around every 8th launch of the timed
    # region: each timed launch pays two event records, ~5.7 us each on the
    # box (~1 % of a C3 step, ~7 % of a 3/8 shard's when every launch is
    # timed: profiles/r02z_event_overhead.txt, profiles/r04r/timeline_*)
    ev_stride = 8
    plan.enable_timing((args.steps + ev_stride - 1) // ev_stride, ev_stride)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    k1_ms, k1_n = plan.kernel_ms()
    k1_name = plan.scan_kernel()
    count = plan.fetch_count()
    parity_ok = True
    res = None
    gpu_trip = plan.fetch_triples() if (rank == 0 and world == 1 and not args.no_cpu_baseline) else None

    # llv entries in this rank's rows (algorithmic bytes)
    host = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        host = esa.download()
        llv_pos = host["llvtab"][:, 0] if len(host["llvtab"]) else np.zeros(0, np.uint64)
        llv_here = int(np.count_nonzero((llv_pos >= begin - 1) & (llv_pos <= end)))
        del llv_pos
    elif use64:
        llv_here = int(esa.numllv)        # the range build holds exactly these rows
    else:
        llv_pos = esa.download()["llvtab"][:, 0] if esa.numllv else np.zeros(0, np.uint64)
        llv_here = int(np.count_nonzero((llv_pos >= begin - 1) & (llv_pos <= end)))
    rows = end - begin + 1
    # 2 B per suffix row (LCP + BWT byte) + 16 B per .llv entry
    # in range + 16 B per emitted interval record (K1's output)
    alg_bytes = 2 * rows + 16 * llv_here + 16 * plan.fetch_count()

    # what the collective layer saw (N > 1): backend, world size, the number
    # of ranks one all-reduce of ones counts over the step's backend, and
    # each rank's device (the driver's SCALE line can be checked for "RCCL
    # saw N ranks on N devices")
    dist_info = None
    if dist:
        dev_t = "cpu" if staged else "cuda"
        ones = torch.ones(1, dtype=torch.int64, device=dev_t)
        dist.all_reduce(ones)
        props = torch.cuda.get_device_properties(local)
        mine_dev = torch.tensor([local, int(getattr(props, "pci_bus_id", -1))], dtype=torch.int64,
                                device=dev_t)
        all_dev = torch.zeros(2 * world, dtype=torch.int64, device=dev_t)
        dist.all_gather_into_tensor(all_dev, mine_dev)
        ad = all_dev.cpu().tolist()
        dist_info = {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                     "allreduce_ranks": int(ones.item()),
                     "rank_devices": [{"rank": r, "local_device": ad[2 * r], "pci_bus_id": ad[2 * r + 1]}
                                      for r in range(world)],
                     "distinct_devices": len({ad[2 * r + 1] for r in range(world)}),
                     "one_gpu_rehearsal": bool(args.one_gpu)}

    stats = torch.tensor([elapsed, float(count), k1_ms / max(k1_n, 1)], dtype=torch.float64,
                         device="cpu" if staged else "cuda")
    if dist:
        mx = stats.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        tot = stats.clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        elapsed, k1_avg_ms = float(mx[0]), float(mx[2])
        count = int(tot[1])
    else:
        k1_avg_ms = float(stats[2])
    ms_per_step = elapsed * 1e3 / args.steps
    value = N / (elapsed / args.steps)
    achieved = alg_bytes / (k1_avg_ms * 1e-3) / 1e9

    # HBM traffic of K1 from the committed PMC profile of this config, used
    # only when that profile was taken on this very build of the scan kernels
    # (gt_smax_build_id stamped by tools/rocpd_summary.py) and config
    traffic = None
    pmc_src = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_%s_n%d.json" % (args.config, world))
    if os.path.exists(pmc_path) and not args.bases and not args.minlen:
        with open(pmc_path) as fh:
            pmc = json.load(fh)
        bid = G.build_id()
        if pmc.get("build_id") == bid and pmc.get("config") == args.config:
            traffic = pmc.get("hbm_bytes_per_launch")
            pmc_src = "%s (build %s)" % (os.path.relpath(pmc_path, ROOT), bid)
        else:
            pmc_src = ("%s not used: taken on build %s / config %s, this run is build %s"
                       % (os.path.relpath(pmc_path, ROOT), pmc.get("build_id"), pmc.get("config"),
                          bid))
    # a per-pass stream (LCP byte + 2-plane BWT = 1.25 B/row, 1.5 B/row with
    # GT_SMAX_BW2=0, + .llv) that fits the 256 MiB Infinity Cache is re-read
    # from it on every pass, not from HBM (MI355X_MICROARCH.md "Infinity
    # Cache"): no HBM fraction is quoted then
    per_row4 = 6 if os.environ.get("GT_SMAX_BW2", "1") == "0" else 5
    stream_bytes = rows * per_row4 // 4 + 16 * llv_here
    in_mall = world == 1 and stream_bytes < (256 << 20)

    # N > 1 parity: every rank's stitched records gathered to rank 0 (padded
    # all-gather over the same backend as the boundary exchange), compared
    # bit for bit with the all-core oracle over the WHOLE table, which rank 0
    # builds after the timed region (no rank holds it during the run)
    dist_parity = None
    if world > 1 and not args.no_parity:
        mine = plan.fetch_triples().view(np.int64).reshape(-1)
        plan.close()
        plan = None
        esa.release()
        esa = None
        dev = "cpu" if staged else "cuda"
        cnts = torch.zeros(world, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(cnts, torch.tensor([len(mine)], dtype=torch.int64, device=dev))
        kmax = max(int(cnts.max()), 1)
        buf = torch.zeros(kmax, dtype=torch.int64, device=dev)
        buf[:len(mine)] = torch.from_numpy(mine).to(dev)
        gathered = torch.zeros(kmax * world, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(gathered, buf)
        del buf, mine
        if rank == 0:
            try:
                g = gathered.cpu().numpy()
                got = np.concatenate([g[r * kmax: r * kmax + int(cnts[r])] for r in range(world)])
                got = got.view(np.uint64).reshape(-1, 3)
                del g
                import oracle_lib  # noqa: E402  (tests/: the checker only)
                t0 = time.time()
                text = G.synth_genome(cfg["kind"], cfg["bases"], cfg["seed"], threads=16)
                if n + 1 >= 2 ** 32 or args.esa64:
                    full = G.DeviceEsa64(text, device=local, row_lo=0, row_hi=n + 1)
                else:
                    full = G.DeviceEsa(text, device=local, keep_suftab=False)
                del text
                ht = full.download()
                full.release()
                threads = max(1, min(len(os.sched_getaffinity(0)), args.cpu_threads))
                want = oracle_lib.linsmax(ht["lcptab"], ht["llvtab"], ht["bwttab"], N, minlen,
                                          threads=threads)
                del ht
                dist_parity = bool(np.array_equal(got, want))
                log("parity (%d ranks): %d gathered records %s the whole-table oracle's %d (%.1fs)"
                    % (world, len(got), "equal" if dist_parity else "DIFFER from", len(want),
                       time.time() - t0))
                if not dist_parity:
                    parity_ok = False
                del got, want
            except Exception as ex:  # noqa: BLE001  (e.g. host memory for the whole table)
                log("rank 0: whole-table parity check could not run: %r" % (ex,))
                dist_parity = False
                parity_ok = False
        del gathered

    cpu = None
    sample_full = False
    if host is not None:
        import oracle_lib  # noqa: E402  (tests/: the checker, CPU baseline leg only)
        # parity: the all-core oracle scan (orc_linsmax_mt, row ranges per
        # pthread, output identical to orc_linsmax) over ALL rows against the
        # timed path's records, bit for bit
        aff = len(os.sched_getaffinity(0))
        threads = max(1, min(aff, args.cpu_threads))
        log("parity: oracle linsmax over all %d rows (%d threads)" % (N, threads))
        t0 = time.perf_counter()
        res = oracle_lib.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], N, minlen,
                                 threads=threads)
        t_mt = time.perf_counter() - t0
        sample_full = True
        if not np.array_equal(gpu_trip, res):
            log("FAIL: GPU (%d intervals) differs from the CPU oracle (%d)"
                % (len(gpu_trip), len(res)))
            parity_ok = False
        else:
            log("GPU interval array equals the CPU oracle's (%d intervals)" % len(res))
        # the single-core baseline on a bounded sample of the same rows
        sample = min(N, args.cpu_sample)
        log("cpu baseline: oracle linsmax over %d rows (1 core)" % sample)
        t0 = time.perf_counter()
        res1 = oracle_lib.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], sample, minlen)
        t_cpu = time.perf_counter() - t0
        if sample == N and not np.array_equal(res1, res):
            log("FAIL: single-core CPU scan (%d intervals) != all-core (%d)" % (len(res1), len(res)))
            parity_ok = False
        del res1
        cpu = {"value": sample / t_cpu, "unit": "suffix-positions/s", "cores": 1, "kind": "port",
               "sample": "oracle orc_linsmax (single core, -O3) over suffix rows [0,%d) of the same "
                         "tables: %.2fs" % (sample, t_cpu)}
        cpu.update(host_cpu())
        # the reference's own algorithm, single core: the bottom-up stack walk
        # of src/match/esa-bottomup.c:116-273 with a smax visitor, reading the
        # tables as the sequential reader hands them out (orc_bottomup_smax_
        # tables) -- the traversal the GPU path replaces -- on a bounded
        # prefix of the rows
        sb = min(N, args.cpu_sample_bottomup)
        log("cpu anchor: bottom-up stack walk over %d rows (1 core)" % sb)
        t0 = time.perf_counter()
        rb = oracle_lib.bottomup_smax_tables(host["lcptab"], host["llvtab"], host["bwttab"], sb,
                                             minlen, cap=max(16, len(res) + 16))
        t_bu = time.perf_counter() - t0
        if sb == N and not np.array_equal(rb, res):
            log("FAIL: bottom-up CPU walk (%d intervals) != linear scan (%d)" % (len(rb), len(res)))
            parity_ok = False
        del rb
        cpu["reference_algorithm_1core"] = {
            "value": sb / t_bu, "cores": 1, "seconds": round(t_bu, 3),
            "sample": "oracle orc_bottomup_smax_tables (the esa-bottomup.c:116-273 stack walk with "
                      "a smax visitor, single core) over suffix rows [0,%d)" % sb}
        cpu["all_cores"] = {"value": N / t_mt, "cores": threads, "seconds": round(t_mt, 3),
                            "sample": "orc_linsmax_mt (pthreads, equal row ranges) over all rows"}
        if aff > threads:
            # every CPU of the affinity mask (the container's quota may be
            # lower: cgroup_cpus); same output as the 16-thread scan
            t0 = time.perf_counter()
            ra = oracle_lib.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], N, minlen,
                                    threads=aff)
            t_aff = time.perf_counter() - t0
            if not np.array_equal(ra, res):
                log("FAIL: %d-thread CPU scan differs" % aff)
                parity_ok = False
            del ra
            cpu["all_affinity_cores"] = {
                "value": N / t_aff, "cores": aff, "seconds": round(t_aff, 3),
                "sample": "orc_linsmax_mt over all rows, one thread per CPU of the affinity mask"}
        cpu["cgroup_cpus"] = cgroup_cpus()

    # end-to-end through the drop-in boundary (host tables in memory -> H2D
    # -> plan -> K1..K3 -> D2H of the (lcp, lb, rb) list): reported beside
    # `value`, never as it.  "cold": the first call in a fresh process
    # (bin/gt-smax-e2e, a C program linking only libgtsmax_hip.so: HIP
    # runtime not initialised, nothing cached), the way one `gt repfind -smax`
    # process meets it (src/tools/gt_repfind.c:553-562); "warm": a call in
    # this process after the timed passes (device cache, pinned ring and code
    # objects ready)
    e2e = None
    if host is not None and not args.no_end_to_end:
        plan.close()
        plan = None
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        iv = G.enumerate_smax(host["lcptab"], host["llvtab"], host["bwttab"], n, N, minlen, 1)
        t_e2e = time.perf_counter() - t0
        if res is not None and not np.array_equal(iv, res):
            log("FAIL: end-to-end result (%d intervals) differs from the CPU oracle (%d)"
                % (len(iv), len(res)))
            parity_ok = False
        path = ("gt_smax_hip_enumerate_to_buffer: pageable host .lcp/.bwt/.llv -> H2D "
                "(.bwt packed to its two code planes + the groups holding a special row during the "
                "staged fill, u64 groups rebuilt on the device) -> plan (llv index) -> "
                "K1..K3 -> D2H of %d (lcp,lb,rb) triples" % len(iv))
        del iv

        def vs(t):
            if not cpu:
                return None
            d = {k: (N / t) / cpu[k]["value"] for k in
                 ("reference_algorithm_1core", "all_cores", "all_affinity_cores") if k in cpu}
            d["linsmax_1core"] = (N / t) / cpu["value"]
            return d
        warm = {"value": N / t_e2e, "unit": "suffix-positions/s", "seconds": round(t_e2e, 4),
                "process": "this process, after the timed passes", "vs_cpu": vs(t_e2e)}
        # the fresh process meets an otherwise idle device: this process's
        # tables and caches go back first (a child creating its HIP context
        # beside a process holding ~20 GB took its first stream 100 ms
        # instead of 22, profiles/r04q vs r04z)
        if esa is not None:
            esa.release()
            esa = None
        G.release_cache()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        cold = cold_e2e(G, host, n, N, minlen, res, log)
        if cold is not None:
            if not cold.pop("parity_ok"):
                parity_ok = False
            cold["vs_cpu"] = vs(cold["seconds"])
            if cold.get("second_call_s"):
                cold["second_call_vs_cpu"] = vs(cold["second_call_s"])
        # a second fresh process: the first one after this process's GPU work
        # created its HIP context's first stream in ~160 ms, later ones in
        # ~22 ms (profiles/r04y, r05f); both are reported
        cold2 = cold_e2e(G, host, n, N, minlen, res, log) if cold is not None else None
        if cold2 is not None:
            if not cold2.pop("parity_ok"):
                parity_ok = False
            cold2["vs_cpu"] = vs(cold2["seconds"])
            cold2.pop("second_call_s", None)
            cold2.pop("phases_second_call", None)
        # a third fresh process with the runner's warm-up (gt_smax_hip_prepare)
        # issued before it reads the tables: the first call's fixed costs
        # (contexts, pinned ring, first allocations) overlap the table read
        cold3 = cold_e2e(G, host, n, N, minlen, res, log, prepared=True) if cold is not None else None
        if cold3 is not None:
            if not cold3.pop("parity_ok"):
                parity_ok = False
            cold3["vs_cpu"] = vs(cold3["seconds"])
            cold3.pop("second_call_s", None)
            cold3.pop("phases_second_call", None)
        e2e = {"path": path, "cold": cold, "cold_next_process": cold2, "cold_prepared": cold3,
               "warm": warm}

    if dist:
        # every rank learns rank 0's verdict, so all of them leave through the
        # barrier and the teardown below instead of waiting in a collective
        flag = torch.tensor([1 if parity_ok else 0], dtype=torch.int64,
                            device="cpu" if staged else "cuda")
        dist.broadcast(flag, 0)
        parity_ok = bool(int(flag.item()))
    if not parity_ok:
        if rank == 0:
            log("parity failure: no bench line")
        if plan is not None:
            plan.close()
        if esa is not None:
            esa.release()
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        sys.exit(1)
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "suffix-positions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": cfg["workload"], "minlen": minlen, "totallength": n,
                       "nonspecials": N,
                       # N > 1: the range build holds rank 0's rows only
                       ("llv_entries" if world == 1 else "llv_entries_rank0_rows"): numllv,
                       "global_batch": N,
                       "parallelism": "sa-range-shard x%d + %s all-gather stitch"
                       % (world, "RCCL" if args.dist_backend == "nccl" else "gloo (rehearsal)")
                       if world > 1 else "single GPU"},
            "smax_intervals": count,
            "supermax_repeats_per_s": count / (elapsed / args.steps),
            "roofline": {"bound": "mall" if in_mall else "hbm", "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         # a stream resident in the Infinity Cache is not an
                         # HBM utilisation: no fraction is quoted for it
                         "frac": None if in_mall else achieved / HBM_PEAK_GBS,
                         "stream_bytes_per_pass": stream_bytes,
                         "traffic": traffic,
                         "kernel": k1_name, "kernel_avg_ms": k1_avg_ms,
                         "kernel_timed_launches": "%d of %d (HIP events on every %dth)"
                                                  % (k1_n, args.steps, ev_stride),
                         "algorithmic_bytes_per_launch": alg_bytes,
                         # the same kernel priced by the HBM bytes it really moves
                         # (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH §HBM)
                         "achieved_by_traffic": (traffic / (k1_avg_ms * 1e-3) / 1e9
                                                 if traffic else None),
                         "frac_by_traffic": (traffic / (k1_avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
                                             if traffic and not in_mall else None),
                         "traffic_source": pmc_src},
            "parity": ("bit-exact vs CPU oracle (plan records%s)" % (" + end-to-end" if e2e else "")
                       if res is not None and sample_full else
                       "bit-exact vs CPU oracle (all %d ranks' stitched records gathered to rank 0 "
                       "vs the all-core oracle over the whole table)" % world
                       if dist_parity else "not checked in this run"),
            "cpu_baseline": cpu,
            "end_to_end": e2e,
            "dist": dist_info,
            "setup_s": {"genome": round(t_gen, 2), "gpu_esa_build": round(t_esa, 2),
                        "builder": builder},
            # plan creation over the resident tables, outside the timed steps
            "plan_ms": round(t_plan * 1e3, 3),
            "plan_ms_warm": round(t_plan_warm * 1e3, 3),
            # untimed full passes before the warmup steps (clock ramp)
            "priming": {"passes": n_prime, "seconds": round(t_prime, 3)},
            "bwt_input": ("byte BWT, packed at plan time" if args.byte_bwt else
                          "packed bit planes (0.5 B/row) emitted by the GPU ESA builder"),
        }
        print(json.dumps(out), flush=True)
    if plan is not None:
        plan.close()
    if esa is not None:
        esa.release()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    main()

"""GPU checks of the host runtime (csrc/smax_runtime.cpp) and of the packed
BWT input form (GT_SMAX_PK_GROUPS, include/gt_smax_hip.h):

  - the GPU ESA builder's packed BWT equals the numpy restatement of the
    layout over its own byte BWT;
  - a plan over the builder's packed BWT, a plan packing the byte BWT itself
    and the CPU oracle give the same interval arrays;
  - the host-table entry point (gt_smax_hip_enumerate_to_buffer) with the
    BWT packed during staging, with the byte fallback, with shards > devices,
    and through the RCCL all-gather (GT_SMAX_FORCE_RCCL: a one-rank
    communicator on the single GPU) equals the oracle;
  - repeated calls on the cached buffers, and after gt_smax_release_cache.
"""
import os

import numpy as np
import pytest

import genometools_smax_amd as G
import oracle_lib as O
from conftest import oracle_esa

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def human10():
    text = G.synth_genome("human", 10_000_000, 7, threads=8)
    esa = G.DeviceEsa(text, device=0)
    host = esa.download()
    yield esa, host
    esa.release()


def test_builder_packed_bwt_matches_layout(human10):
    esa, host = human10
    got = esa.packed_bwt()
    want, dna = O.pack_bwt_ref(host["bwttab"])
    assert dna
    assert np.array_equal(got, want)


def test_plan_packed_and_byte_bwt_agree(human10):
    esa, host = human10
    want = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], esa.nonspecials, 20)
    for packed in (True, False):
        p = esa.plan(20, packed=packed)
        p.run()
        got = p.fetch_triples()
        p.close()
        assert np.array_equal(got, want), (packed, len(got), len(want))


def test_run_in_two_parts(human10):
    """gt_smax_plan_run_part: scan then compaction equals plan_run, repeated
    (each run's compaction resets the next run's deferral state); the
    boundary record is final after part 0 (bench.py starts the all-gather
    there, beside the compaction)."""
    import torch
    esa, host = human10
    N = esa.nonspecials
    want = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], N, 20)

    def bnd(plan):
        t = torch.zeros(G.BOUNDARY_BYTES, dtype=torch.uint8, device="cuda")
        plan.copy_boundary(t.data_ptr())
        torch.cuda.synchronize()
        return t.cpu().numpy()

    for begin, end in ((1, N), (1, N // 2), (N // 3, N)):
        p = esa.plan(20, begin, end)
        ref = esa.plan(20, begin, end)
        ref.run()
        ref_trip, ref_bnd = ref.fetch_triples(), bnd(ref)
        if (begin, end) == (1, N):
            assert np.array_equal(ref_trip, want)
        bt = p.boundary_tensor()           # zero-copy view (bench.py's send buffer)
        assert bt.data_ptr() == p.boundary_ptr and bt.numel() == G.BOUNDARY_BYTES
        for _ in range(3):
            p.run_part(0)
            assert np.array_equal(bnd(p), ref_bnd)
            torch.cuda.synchronize()
            assert np.array_equal(bt.cpu().numpy(), ref_bnd)
            p.run_part(1)
            assert np.array_equal(p.fetch_triples(), ref_trip)
        with pytest.raises(G.SmaxError):
            p.run_part(2)
        p.close()
        ref.close()


def _host_call(e, minlen, shards, **env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return G.enumerate_smax(e.lcpbytes, e.llv, e.bwt, e.n, e.nonspecials, minlen, shards)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("shards", [1, 3])
@pytest.mark.parametrize("env", [{}, {"GT_SMAX_BYTE_BWT": 1}, {"GT_SMAX_FORCE_RCCL": 1}])
def test_host_entry_variants(shards, env):
    e = oracle_esa("at1MB")
    want = O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, 20)
    got = _host_call(e, 20, shards, **env)
    assert np.array_equal(got, want), (shards, env, len(got), len(want))


@pytest.mark.parametrize("shards", [7, 8])
def test_more_shards_than_devices_through_rccl(shards):
    """num_gpus = 7 / 8 on one device through the in-library RCCL path (a
    one-rank communicator: GT_SMAX_FORCE_RCCL), C4's shard count included."""
    e = oracle_esa("at1MB")
    want = O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, 8)
    got = _host_call(e, 8, shards, GT_SMAX_FORCE_RCCL=1)
    assert np.array_equal(got, want)


def test_eight_shards_rccl_human(human10):
    """The C-ABI with num_gpus = 8 over a 10 Mbp human-like index on one
    device through the RCCL all-gather path: eight shards' boundary records
    exchanged, stitched, bit-exact with the oracle."""
    esa, host = human10
    want = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], esa.nonspecials, 20)
    old = os.environ.get("GT_SMAX_FORCE_RCCL")
    os.environ["GT_SMAX_FORCE_RCCL"] = "1"
    try:
        got = G.enumerate_smax(host["lcptab"], host["llvtab"], host["bwttab"], esa.totallength,
                               esa.nonspecials, 20, 8)
    finally:
        if old is None:
            os.environ.pop("GT_SMAX_FORCE_RCCL", None)
        else:
            os.environ["GT_SMAX_FORCE_RCCL"] = old
    assert np.array_equal(got, want)


def test_repeated_calls_and_cache_release(human10):
    esa, host = human10
    args = (host["lcptab"], host["llvtab"], host["bwttab"], esa.totallength, esa.nonspecials, 20)
    want = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], esa.nonspecials, 20)
    for _ in range(3):
        assert np.array_equal(G.enumerate_smax(*args, 1), want)
    G.release_cache()
    assert np.array_equal(G.enumerate_smax(*args, 2), want)
    G.release_cache()


def test_timing_stride(human10):
    """gt_smax_plan_timing_stride: K1 events around every stride-th run only;
    the read covers exactly those runs."""
    esa, _ = human10
    p = esa.plan(20)
    for stride, runs, want in ((1, 5, 5), (4, 10, 3), (4, 12, 3), (3, 1, 1)):
        p.enable_timing(16, stride)
        for _ in range(runs):
            p.run()
        ms, n = p.kernel_ms()
        assert n == want, (stride, runs, n)
        assert ms > 0.0
    p.close()


@pytest.mark.parametrize("odd", [1, 3])
def test_timing_reset_keeps_block_sums(human10, odd):
    """The timing calls reset the run counter; the block-sum buffer a pass
    adds into must not follow it (after an odd number of runs the
    next pass added into the buffer the last pass filled).  Odd runs, then
    enable_timing, then more runs -- whole and split -- each checked against
    the oracle, whole table and a middle shard."""
    esa, host = human10
    N = esa.nonspecials
    want = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], N, 20)
    p = esa.plan(20)
    q = esa.plan(20, N // 3, 2 * N // 3)
    r = esa.plan(20, N // 3, 2 * N // 3)
    r.run()
    ref = r.fetch_triples()
    for _ in range(odd):
        p.run()
        q.run()
    for stride in (1, 4):
        p.enable_timing(8, stride)
        q.enable_timing(8, stride)
        for k in range(3):
            if k == 1:
                p.run_part(0)
                p.enable_timing(8, stride)    # a reset between the two parts
                p.run_part(1)
            else:
                p.run()
            q.run()
            assert np.array_equal(p.fetch_triples(), want), (odd, stride, k)
            assert np.array_equal(q.fetch_triples(), ref), (odd, stride, k)
    for x in (p, q, r):
        x.close()


@pytest.mark.parametrize("bw2", ["0", "1"])
@pytest.mark.parametrize("nt", ["0", "1"])
@pytest.mark.parametrize("dense", ["0", "1"])
def test_window_stream_policy(human10, nt, dense, bw2):
    """Both window-stream policies of K1 (GT_SMAX_NT; the plan picks nt by
    shard size, 2-plane windows only), both K1 variants and both BWT window
    forms (GT_SMAX_BW2: the 2-plane stream, windows with a special BWT row
    left to K1b; or the u64 groups) give the oracle's records, whole table
    and a middle shard's plan run (against the plain-policy plan); the plan
    launches the variant the switches name."""
    esa, host = human10
    N = esa.nonspecials
    want = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], N, 20)
    old = {k: os.environ.get(k) for k in ("GT_SMAX_NT", "GT_SMAX_DENSE", "GT_SMAX_BW2")}
    os.environ.update(GT_SMAX_NT=nt, GT_SMAX_DENSE=dense, GT_SMAX_BW2=bw2)
    try:
        p = esa.plan(20)
        q = esa.plan(20, N // 3, 2 * N // 3)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    name = ("smax_scan_kernel" + ("_b2" if bw2 == "1" else "") + ("_dense" if dense == "1" else "")
            + ("_nt" if nt == "1" and bw2 == "1" else ""))
    assert p.scan_kernel() == name and q.scan_kernel() == name, (p.scan_kernel(), name)
    p.run()
    assert np.array_equal(p.fetch_triples(), want)
    r = esa.plan(20, N // 3, 2 * N // 3)
    q.run()
    r.run()
    assert np.array_equal(q.fetch_triples(), r.fetch_triples())
    for x in (p, q, r):
        x.close()


@pytest.mark.parametrize("waves", ["4", "8"])
def test_k1b_workgroup_widths(human10, waves):
    """K1b with 4 or 8 waves per tile workgroup (the plan picks 8 when the
    launch fits one generation of them; GT_SMAX_K1B_WAVES forces either):
    the oracle's records, whole table and a middle shard, two consecutive
    runs each (the block-sum workgroups then sum 4 or 8 blocks)."""
    esa, host = human10
    N = esa.nonspecials
    want = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], N, 20)
    old = os.environ.get("GT_SMAX_K1B_WAVES")
    os.environ["GT_SMAX_K1B_WAVES"] = waves
    try:
        p = esa.plan(20)
        q = esa.plan(20, N // 3, 2 * N // 3)
    finally:
        if old is None:
            os.environ.pop("GT_SMAX_K1B_WAVES", None)
        else:
            os.environ["GT_SMAX_K1B_WAVES"] = old
    r = esa.plan(20, N // 3, 2 * N // 3)
    assert p.k1b_waves() == int(waves) and q.k1b_waves() == int(waves)
    for _ in range(2):
        p.run()
        assert np.array_equal(p.fetch_triples(), want)
        q.run()
        r.run()
        assert np.array_equal(q.fetch_triples(), r.fetch_triples())
    for x in (p, q, r):
        x.close()


def test_block_sums_in_k1b_launch(human10):
    """K3's block sums added up by K1b's last workgroups (two buffers: each
    run adds into one, its K3 clears the other): the oracle's records over
    five consecutive runs (both buffers twice), split runs included, whole
    table and a middle shard."""
    esa, host = human10
    N = esa.nonspecials
    want = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], N, 20)
    p = esa.plan(20)
    q = esa.plan(20, N // 3, 2 * N // 3)
    r = esa.plan(20, N // 3, 2 * N // 3)
    r.run()
    ref = r.fetch_triples()
    for k in range(5):
        if k == 2:
            p.run_part(0)
            p.run_part(1)
        else:
            p.run()
        q.run()
        assert np.array_equal(p.fetch_triples(), want), k
        assert np.array_equal(q.fetch_triples(), ref), k
    for x in (p, q, r):
        x.close()


@pytest.mark.parametrize("split", ["1", "3", "8"])
def test_compact_split_blocks(human10, split):
    """K3 with `split` workgroups per block of 256 tiles, each copying its
    share of the block's records (GT_SMAX_K3_SPLIT): the oracle's records,
    whole table and a middle shard, over repeated runs."""
    esa, host = human10
    N = esa.nonspecials
    want = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], N, 20)
    old = os.environ.get("GT_SMAX_K3_SPLIT")
    os.environ["GT_SMAX_K3_SPLIT"] = split
    try:
        p = esa.plan(20)
        q = esa.plan(20, N // 3, 2 * N // 3)
    finally:
        if old is None:
            os.environ.pop("GT_SMAX_K3_SPLIT", None)
        else:
            os.environ["GT_SMAX_K3_SPLIT"] = old
    r = esa.plan(20, N // 3, 2 * N // 3)
    r.run()
    for _ in range(3):
        p.run()
        q.run()
        assert np.array_equal(p.fetch_triples(), want)
        assert np.array_equal(q.fetch_triples(), r.fetch_triples())
    for x in (p, q, r):
        x.close()


def test_run_part_order_enforced(human10):
    """Part 1's K3 resets the state the next part 0 starts from: a second
    part 0 before part 1, or a part 1 with no part 0 pending, is refused
    (include/gt_smax_hip.h, gt_smax_plan_run_part) and the plan stays usable."""
    esa, host = human10
    want = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], esa.nonspecials, 20)
    p = esa.plan(20)
    with pytest.raises(G.SmaxError):
        p.run_part(1)
    p.run_part(0)
    with pytest.raises(G.SmaxError):
        p.run_part(0)
    p.run_part(1)
    assert np.array_equal(p.fetch_triples(), want)
    p.run()
    assert np.array_equal(p.fetch_triples(), want)
    p.close()


def test_close_in_flight_then_reuse(human10):
    """A plan closed right after run() with no synchronisation hands its
    buffers back to the caching pool only once its kernels have finished:
    new plans and an ESA build that take the same blocks at once still give
    the oracle's records."""
    esa, host = human10
    N = esa.nonspecials
    want = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], N, 20)
    for _ in range(3):
        p = esa.plan(20)
        for _ in range(4):
            p.run()
        p.close()                       # K1..K3 may still be running
        q = esa.plan(20)
        small = G.DeviceEsa(G.synth_genome("uniform", 1_000_000, 3, threads=4), device=0)
        q.run()
        assert np.array_equal(q.fetch_triples(), want)
        q.close()
        small.release()


def test_plan_on_own_stream_then_delete(human10):
    """A plan run on a stream of the caller's (alive until the delete, as
    gt_smax_hip.h requires), fetched, run again and deleted with the run in
    flight: the fence recorded at delete keeps the buffers until then."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    esa, host = human10
    want = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], esa.nonspecials, 20)
    for _ in range(2):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(s)) == 0
        p = esa.plan(20)
        for _ in range(3):
            p.run(s.value)
        got = p.fetch_triples()          # waits on the plan's streams
        p.run(s.value)
        p.close()                        # fence recorded on s, nothing waits
        q = esa.plan(20)
        q.run()
        assert np.array_equal(q.fetch_triples(), want)
        q.close()
        assert hip.hipStreamDestroy(s) == 0
        assert np.array_equal(got, want)


@pytest.mark.skipif(G.device_count() < 2, reason="needs >= 2 visible GPUs")
@pytest.mark.parametrize("shards", [2, 3, 8])
def test_host_entry_across_devices(human10, shards):
    """num_gpus > 1 with several devices visible: one host thread per device
    and the in-library RCCL all-gather (ncclCommInitAll) between them."""
    esa, host = human10
    want = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], esa.nonspecials, 20)
    got = G.enumerate_smax(host["lcptab"], host["llvtab"], host["bwttab"], esa.totallength,
                           esa.nonspecials, 20, shards)
    assert np.array_equal(got, want)


DIAG_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "genometools_smax_amd", "lib", "diag", "libgtsmax_hip.so")


@pytest.mark.skipif(not os.path.exists(DIAG_LIB), reason="diagnostic build not present")
def test_diag_build_forces_two_plane_stream():
    """The diagnostic kernel (diag build only) streams the 2-plane BWT:
    GT_SMAX_STAMPS with GT_SMAX_BW2=0 must still plan the 2-plane buffers
    (it once passed a null plane pointer to the diagnostic kernel), and the
    records equal the oracle's.  Own process: the library is chosen at load."""
    import subprocess
    import sys
    code = r'''
import numpy as np, sys
sys.path.insert(0, "tests")
import genometools_smax_amd as G, oracle_lib as O
from conftest import oracle_esa
e = oracle_esa("at1MB")
for m in (5, 20, 256):
    got = G.enumerate_smax(e.lcpbytes, e.llv, e.bwt, e.n, e.nonspecials, m, 2)
    assert np.array_equal(got, O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, m)), m
print("diag ok")
'''
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GT_SMAX_LIB=DIAG_LIB, GT_SMAX_BW2="0", GT_SMAX_STAMPS="1")
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and "diag ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("fail_at", [1, 2])
def test_pin_failure_shrinks_ring(fail_at):
    """A staging chunk whose pinning fails (GT_SMAX_PIN_FAIL_AT: chunk i and
    later report hipErrorOutOfMemory) shrinks the device's upload/download
    ring to the chunks pinned before it; the calls still succeed, again and
    again, with 1 MiB chunks so that every transfer spans many of them.  Own
    process: the ring is created once per device."""
    import subprocess
    import sys
    code = r'''
import numpy as np, sys
sys.path.insert(0, "tests")
import genometools_smax_amd as G, oracle_lib as O
from conftest import oracle_esa
e = oracle_esa("at1MB")
for shards in (1, 2, 1):
    got = G.enumerate_smax(e.lcpbytes, e.llv, e.bwt, e.n, e.nonspecials, 5, shards)
    assert np.array_equal(got, O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, 5)), shards
print("pin ok")
'''
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GT_SMAX_PIN_FAIL_AT=str(fail_at), GT_SMAX_STAGE_MB="1")
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and "pin ok" in r.stdout, r.stdout + r.stderr


def test_prepare_then_calls():
    """gt_smax_hip_prepare (asynchronous warm-up) ahead of host-table calls:
    the calls wait for it and stay bit-exact, whatever sizes or shard count
    it announced; release_cache waits for a warm-up in flight.  Fresh process
    (the warm-up then creates the contexts), and again in this one."""
    import subprocess
    import sys
    code = r'''
import numpy as np, sys
sys.path.insert(0, "tests")
import genometools_smax_amd as G, oracle_lib as O
from conftest import oracle_esa
e = oracle_esa("at1MB")
want = O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, 12)
G.prepare(e.n, e.nonspecials, 2)
assert np.array_equal(G.enumerate_smax(e.lcpbytes, e.llv, e.bwt, e.n, e.nonspecials, 12, 2), want)
G.prepare(10 * e.n, 10 * e.nonspecials, 3)          # other sizes: only the cache differs
assert np.array_equal(G.enumerate_smax(e.lcpbytes, e.llv, e.bwt, e.n, e.nonspecials, 12, 1), want)
G.prepare(e.n, e.nonspecials, 1)
G.release_cache()
assert np.array_equal(G.enumerate_smax(e.lcpbytes, e.llv, e.bwt, e.n, e.nonspecials, 12, 1), want)
print("prepare ok")
'''
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "prepare ok" in r.stdout, r.stdout + r.stderr
    e = oracle_esa("at1MB")
    G.prepare(e.n, e.nonspecials, 1)
    got = G.enumerate_smax(e.lcpbytes, e.llv, e.bwt, e.n, e.nonspecials, 20, 1)
    assert np.array_equal(got, O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, 20))


def test_guided_schedule_against_static_grids():
    """K1's guided tile schedule (several generations, per-workgroup table
    with the first tiles' .llv words) against static grids (GT_SMAX_GRID:
    every workgroup strides the whole range), on a table large enough for
    several generations (40 Mbp, ~20 k tiles), whole and a middle shard:
    all equal the oracle's records."""
    text = G.synth_genome("human", 40_000_000, 7)
    esa = G.DeviceEsa(text)
    del text
    host = esa.download()
    N = esa.nonspecials
    want = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], N, 20)
    mid = (N // 3, 2 * N // 3)
    ref_mid = None
    for grid in (None, "6144", "97"):
        old = os.environ.get("GT_SMAX_GRID")
        if grid is not None:
            os.environ["GT_SMAX_GRID"] = grid
        try:
            p = esa.plan(20)
            q = esa.plan(20, *mid)
        finally:
            if old is None:
                os.environ.pop("GT_SMAX_GRID", None)
            else:
                os.environ["GT_SMAX_GRID"] = old
        for _ in range(2):
            p.run()
            assert np.array_equal(p.fetch_triples(), want), grid
            q.run()
            got = q.fetch_triples()
            if ref_mid is None:
                ref_mid = got
            assert np.array_equal(got, ref_mid), grid
        p.close()
        q.close()
    esa.release()


def test_f2_f3_plans_do_not_wait_for_other_streams():
    """The F2 and F3 device entry points are stream-ordered: an F3 plan built
    and its events enqueued on one stream, an F2 plan counted and its total
    read on another, all while a long smax pass runs on a third, return --
    results final -- before that pass does (none of them synchronises the
    device), and their results are bit-exact.  Run in a fresh process
    (tests/stream_order_scenario.py): HIP multiplexes streams onto four
    hardware queues round-robin, and after the other tests' streams the three
    could share one, which serialises them in hardware whatever the library
    does."""
    import json
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "stream_order_scenario.py")],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["waited"] == [], out
    assert out["t_all"] > out["t_calls"]
    assert out["intervals_equal"] and out["events_count_ok"] and out["pairs_equal"], out

"""GPU parity for the generic bottom-up traversal: the
lcp-interval tree computed on the GPU (ANSV searches) and replayed as
GtESAVisitor events must equal, event for event and in order, the oracle's
restatement of gt_esa_bottomup (src/match/esa-bottomup.c:116-273,
orc_bottomup_events) -- leaf edges, branching edges, lcp-intervals, the
firstsucc flags and every father/child field.  The reference's own
lcp-interval test compares its two traversals with each other
(`-enumlcpitvtreeBU` vs `-enumlcpitvtree` on Reads2.fna,
testsuite/gt_suffixerator_include.rb:597-603) and stores no output; the
oracle restates both (orc_bottomup_events, orc_dfs_events) and
tests/test_oracle.py checks that they agree, on Reads2.fna among others.
"""
import numpy as np
import pytest

import genometools_smax_amd as G
import oracle_lib as O
from conftest import oracle_esa

pytestmark = pytest.mark.gpu


def _gpu_events(e, suf_dtype=np.uint64):
    ev = []
    G.esa_bottomup(e.lcpbytes, e.llv, e.suftab.astype(suf_dtype), e.n, e.nonspecials,
                   leaf_edge=lambda f, fd, flb, leaf: ev.append((0, f, fd, flb, leaf, 0, 0)),
                   branching_edge=lambda f, fd, flb, sd, slb, srb:
                   ev.append((1, f, fd, flb, sd, slb, srb)),
                   lcp_interval=lambda l, lb, rb: ev.append((2, 0, l, lb, rb, 0, 0)))
    return np.array(ev, dtype=np.uint64).reshape(-1, 7)


def _want_intervals(ev):
    father = {}
    for r in ev[ev[:, 0] == 1]:
        father[(int(r[4]), int(r[5]))] = (int(r[2]), int(r[3]))
    out = [(int(r[2]), int(r[3]), int(r[4])) + father[(int(r[2]), int(r[3]))]
           for r in ev[ev[:, 0] == 2]]
    return np.array(out, dtype=np.uint64).reshape(-1, 5)


@pytest.mark.parametrize("name", ["Reads2.fna", "Atinsert.fna", "at1MB", "Random.fna",
                                  "TTT-small.fna"])
def test_fixture_event_stream(name):
    e = oracle_esa(name)
    want = O.bottomup_events(e)
    got = _gpu_events(e)
    assert got.shape == want.shape
    assert np.array_equal(got, want)
    itv = G.enumerate_lcp_intervals(e.lcpbytes, e.llv, e.n, e.nonspecials)
    assert np.array_equal(itv, _want_intervals(want))


def test_suftab_4_bytes():
    e = oracle_esa("Atinsert.fna")
    assert np.array_equal(_gpu_events(e, np.uint32), O.bottomup_events(e))


@pytest.mark.parametrize("seed", range(6))
def test_random_texts(seed):
    rng = np.random.default_rng(500 + seed)
    n = int(rng.integers(1, 40000))
    t = rng.integers(0, int(rng.integers(1, 5)), n, dtype=np.uint8)
    if seed % 2:
        t[rng.random(n) < 0.01] = 254
        t[rng.random(n) < 0.005] = 255
    if seed >= 3:                       # long repeats: .llv values
        a = rng.integers(0, 4, 700, dtype=np.uint8)
        t = np.concatenate([t, a, np.array([255], np.uint8), a, a])
    e = O.Esa(t)
    want = O.bottomup_events(e)
    assert np.array_equal(_gpu_events(e), want)
    assert np.array_equal(G.enumerate_lcp_intervals(e.lcpbytes, e.llv, e.n, e.nonspecials),
                          _want_intervals(want))


def test_homopolymer_tiles_overflow_slots():
    """Homopolymer runs give whole tiles of monotone LCP (a run followed by a
    larger symbol: decreasing, every row's PL outside its tile; a run at the
    end of a sequence: increasing, every row's NSE outside): more unresolved
    rows per tile than pass A's slots hold, so pass B scans those tiles."""
    rng = np.random.default_rng(71)
    t = np.concatenate([rng.integers(0, 4, 3000, dtype=np.uint8), np.zeros(5000, np.uint8),
                        np.ones(1, np.uint8), rng.integers(0, 4, 3000, dtype=np.uint8),
                        np.full(4500, 2, np.uint8), np.array([254], np.uint8),
                        rng.integers(0, 4, 2000, dtype=np.uint8), np.full(2500, 3, np.uint8)])
    e = O.Esa(t)
    want = O.bottomup_events(e)
    assert np.array_equal(_gpu_events(e), want)
    assert np.array_equal(G.enumerate_lcp_intervals(e.lcpbytes, e.llv, e.n, e.nonspecials),
                          _want_intervals(want))


def test_callback_stop_and_partial_visitor():
    e = oracle_esa("Atinsert.fna")
    seen = []
    with pytest.raises(G.SmaxError):
        G.esa_bottomup(e.lcpbytes, e.llv, e.suftab, e.n, e.nonspecials,
                       lcp_interval=lambda l, lb, rb: seen.append(lb) or len(seen) >= 5)
    assert len(seen) == 5
    # intervals only (no suftab needed): the lcp-interval callbacks alone
    itv = []
    G.esa_bottomup(e.lcpbytes, e.llv, None, e.n, e.nonspecials,
                   lcp_interval=lambda l, lb, rb: itv.append((l, lb, rb)))
    want = O.bottomup_events(e)
    assert np.array_equal(np.array(itv, dtype=np.uint64), want[want[:, 0] == 2][:, 2:5])


def test_device_resident_tree_and_events():
    # gt_lcpitv_plan_*: tree and event stream built and kept in HBM from a
    # GPU-built index, equal to the oracle's traversal of the same tables
    import torch
    e = oracle_esa("at1MB")
    d = G.DeviceEsa(e.text, keep_suftab=True)
    p = d.lcpitv_plan()
    want = O.bottomup_events(e)
    n_ev = p.num_events()
    assert n_ev == len(want)
    ev = torch.empty(7 * n_ev, dtype=torch.int64, device="cuda")
    p.events(ev.data_ptr())
    torch.cuda.synchronize()
    got = ev.cpu().numpy().view(np.uint64).reshape(-1, 7)
    assert np.array_equal(got, want)
    n, ptr = p.intervals()

    class _View:       # the plan's device records as a torch view (no copy)
        __cuda_array_interface__ = {"shape": (5 * n,), "typestr": "<i8", "data": (ptr, False),
                                    "version": 2}
    itv = torch.as_tensor(_View(), device="cuda").cpu().numpy().view(np.uint64).reshape(-1, 5)
    assert np.array_equal(itv, _want_intervals(want))
    p.close()
    d.release()


NONE = np.uint64(2 ** 64 - 1)


def _run_info_visitor(e):
    """gt_esa_bottomup_info_hip with integer handles: every callback recorded
    as (event record, father handle, son handle), handles 1, 2, ... in
    info_new order, and the handles info_delete received."""
    made, deleted, out = [0], [], []

    def new():
        made[0] += 1
        return made[0]

    G.esa_bottomup_info(e.lcpbytes, e.llv, e.suftab, e.n, e.nonspecials, new, deleted.append,
                        leaf_edge=lambda f, fd, flb, fi, leaf: out.append(((0, f, fd, flb, leaf, 0, 0),
                                                                          fi, 0)),
                        branching_edge=lambda f, fd, flb, fi, sd, slb, srb, si:
                            out.append(((1, f, fd, flb, sd, slb, srb), fi, si)),
                        lcp_interval=lambda lcp, lb, rb, i: out.append(((2, 0, lcp, lb, rb, 0, 0), i, 0)))
    return out, made[0], deleted


@pytest.mark.parametrize("name", ["Atinsert.fna", "at1MB", "Reads2.fna", "TTT-small.fna"])
def test_info_visitor_matches_reference_stack(name):
    """Per-node visitor state (GtESAVisitorInfo, esa_visitor_rep.h:25-67):
    every callback gets the info object the reference's stack slot would
    hand it (orc_bottomup_events_slots: handle = slot + 1, none = 0), the
    objects are created 32 at a time as the stack grows and each is deleted
    once, in slot order, after the traversal (esa-bottomup.c:20-110)."""
    e = oracle_esa(name)
    want_ev, want_sl, nslots = O.bottomup_events_slots(e)
    got, made, deleted = _run_info_visitor(e)
    assert np.array_equal(np.array([g[0] for g in got], dtype=np.uint64).reshape(-1, 7), want_ev)
    handles = np.array([(g[1], g[2]) for g in got], dtype=np.uint64).reshape(-1, 2)
    want_h = np.where(want_sl == NONE, np.uint64(0), want_sl + np.uint64(1))
    want_h[want_ev[:, 0] != 1, 1] = 0          # son handles exist on branching edges only
    assert np.array_equal(handles, want_h)
    assert made == nslots and deleted == list(range(1, nslots + 1))


def test_info_visitor_leaf_counts_deep_stack():
    """A visitor that needs per-node state -- the leaves below each interval,
    accumulated through the info objects (a father pushed into its first
    child's slot inherits the child's count, as the reference hands the
    child's state over) -- reports rb - lb + 1 for every interval; the text
    nests more than 32 intervals (a second chunk of info objects)."""
    rng = np.random.default_rng(17)
    t = np.concatenate([rng.integers(0, 4, 3000, dtype=np.uint8), np.full(150, 3, np.uint8),
                        np.zeros(1, np.uint8), rng.integers(0, 4, 3000, dtype=np.uint8)])
    e = O.Esa(t)
    state, bad, seen = {}, [], [0]

    def leaf(f, fd, flb, fi, leafnumber):
        state[fi] = 1 if f else state[fi] + 1

    def branch(f, fd, flb, fi, sd, slb, srb, si):
        if si == 0:
            assert f == 1 and flb == slb
        elif f:
            state[fi] = state[si]
        else:
            state[fi] += state[si]

    def itv(lcp, lb, rb, i):
        seen[0] += 1
        if state[i] != rb - lb + 1:
            bad.append((lcp, lb, rb))

    made = [0]

    def new():
        made[0] += 1
        return made[0]

    G.esa_bottomup_info(e.lcpbytes, e.llv, e.suftab, e.n, e.nonspecials, new, None, leaf, branch, itv)
    assert made[0] > 32 and seen[0] > 1000
    assert bad == []


# ---------------------------------------- spmitv: a reference golden for F3
# `gt dev sfxmap -spmitv` (src/match/esa-spmitvs.c:25-69) is gt_esa_bottomup
# driving the spmitvs visitor (src/match/esa_spmitvs_visitor.c:59-226); its
# output on Reads2.fna is reference testdata (testdata/Reads2-spmitv.txt,
# testsuite/gt_suffixerator_include.rb:587-592).  Here the GPU traversal
# (gt_esa_bottomup_hip over the index's .lcp/.llv/.suf, the callbacks on
# this thread) drives the same visitor restatement (orc_spmitv) and must
# print the golden byte for byte; on the other fixtures the GPU-driven
# output must equal the oracle-driven one.

def _gpu_spmitv(ix, sep_text):
    ev = _gpu_events_tables(ix.lcptab, ix.llvtab, ix.suftab, ix.totallength, ix.nonspecials)
    return O.spmitv_lines(ev, sep_text, ix.nonspecials)


def _gpu_events_tables(lcptab, llvtab, suftab, n, N):
    ev = []
    G.esa_bottomup(np.asarray(lcptab), np.asarray(llvtab), np.asarray(suftab), n, N,
                   leaf_edge=lambda f, fd, flb, leaf: ev.append((0, f, fd, flb, leaf, 0, 0)),
                   branching_edge=lambda f, fd, flb, sd, slb, srb:
                   ev.append((1, f, fd, flb, sd, slb, srb)),
                   lcp_interval=lambda l, lb, rb: ev.append((2, 0, l, lb, rb, 0, 0)))
    return np.array(ev, dtype=np.uint64).reshape(-1, 7)


def test_spmitv_reads2_golden_from_gpu_traversal(tmp_path):
    import os
    from conftest import GOLDEN
    idx = str(tmp_path / "Reads2.fna")
    O.index_fasta(os.path.join(GOLDEN, "Reads2.fna"), idx)
    ix = G.EsaIndex(idx)
    sep_text = np.zeros(ix.totallength, np.uint8)
    sep_text[ix.separators().astype(np.int64)] = 255
    lines = _gpu_spmitv(ix, sep_text)
    with open(os.path.join(GOLDEN, "Reads2-spmitv.txt")) as fh:
        assert lines == fh.read().splitlines()


@pytest.mark.parametrize("name", ["Atinsert.fna", "at1MB", "Random.fna", "TTT-small.fna"])
def test_spmitv_gpu_equals_oracle(name):
    e = oracle_esa(name)
    want = O.spmitv_lines(O.bottomup_events(e), e.text, e.nonspecials)
    ev = _gpu_events_tables(e.lcpbytes, e.llv, e.suftab, e.n, e.nonspecials)
    assert O.spmitv_lines(ev, e.text, e.nonspecials) == want


def test_spmitv_device_event_stream():
    # the device-resident path: gt_lcpitv_plan_events into HBM (no host
    # callbacks), downloaded and fed to the same visitor
    import torch
    e = oracle_esa("Reads2.fna")
    lcp = torch.from_numpy(np.ascontiguousarray(e.lcpbytes)).cuda()
    llv = torch.from_numpy(np.ascontiguousarray(
        np.vstack([e.llv, np.zeros((1, 2), np.uint64)]).view(np.int64))).cuda()
    suf = torch.from_numpy(e.suftab.view(np.int64)).cuda()
    plan = G.LcpitvPlan(lcp.data_ptr(), llv.data_ptr(), len(e.llv), suf.data_ptr(), 8,
                        e.nonspecials)
    ne = plan.num_events()
    out = torch.zeros(7 * ne, dtype=torch.int64, device="cuda")
    plan.events(out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    plan.close()
    ev = out.cpu().numpy().view(np.uint64).reshape(-1, 7)
    from conftest import GOLDEN
    import os
    with open(os.path.join(GOLDEN, "Reads2-spmitv.txt")) as fh:
        assert O.spmitv_lines(ev, e.text, e.nonspecials) == fh.read().splitlines()

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

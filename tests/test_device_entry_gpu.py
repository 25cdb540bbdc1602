"""The host-table entry points run on the calling thread's current HIP device
and leave it as they found it: smax
(gt_smax_hip_enumerate_to_buffer), maximal pairs
(gt_maxpairs_hip_enumerate_to_buffer, the reference's default runner,
src/match/esa-maxpairs.c:476-520), the lcp-interval tree
(gt_lcpitv_hip_enumerate_to_buffer) and the visitor replay
(gt_esa_bottomup_hip).  hipGetDevice is read straight from the HIP runtime
(ctypes on libamdhip64), not through torch's own device bookkeeping.  The
device-1 variants need a second GPU and are skipped on one.
"""
import ctypes

import numpy as np
import pytest

import genometools_smax_amd as G
import oracle_lib as O
from conftest import oracle_esa

pytestmark = pytest.mark.gpu

_hip = None


def _hiprt():
    global _hip
    if _hip is None:
        for name in ("libamdhip64.so", "libamdhip64.so.7", "libamdhip64.so.6",
                     "/opt/rocm/lib/libamdhip64.so"):
            try:
                _hip = ctypes.CDLL(name)
                break
            except OSError:
                continue
        assert _hip is not None, "libamdhip64 not found"
    return _hip


def _get_device():
    d = ctypes.c_int(-1)
    assert _hiprt().hipGetDevice(ctypes.byref(d)) == 0
    return d.value


def _set_device(k):
    assert _hiprt().hipSetDevice(ctypes.c_int(k)) == 0


def _calls(e):
    """(name, thunk, check) for each host-table entry point."""
    smax_want = O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, 20)
    mp_want = O.maxpairs(e, 20)
    itv_want = O.lcp_intervals(e.lcpbytes, e.llv, e.nonspecials, 2 * e.n + 16)
    ev = O.bottomup_events(e)
    pops = ev[ev[:, 0] == 2][:, 2:5]            # the lcp_interval callbacks, in order
    events = []

    def bottomup():
        events.clear()
        G.esa_bottomup(e.lcpbytes, e.llv, e.suftab, e.n, e.nonspecials,
                       lcp_interval=lambda lcp, lb, rb: events.append((lcp, lb, rb)) or 0)
        return np.array(events, dtype=np.uint64).reshape(-1, 3)

    return [
        ("smax", lambda: G.enumerate_smax(e.lcpbytes, e.llv, e.bwt, e.n, e.nonspecials, 20, 1),
         lambda got: np.array_equal(got, smax_want)),
        ("smax_2_shards", lambda: G.enumerate_smax(e.lcpbytes, e.llv, e.bwt, e.n, e.nonspecials, 20, 2),
         lambda got: np.array_equal(got, smax_want)),
        ("maxpairs", lambda: G.enumerate_maxpairs(e.lcpbytes, e.llv, e.bwt, e.suftab, e.n,
                                                  e.nonspecials, 20),
         lambda got: np.array_equal(got, mp_want)),
        ("lcp_intervals", lambda: G.enumerate_lcp_intervals(e.lcpbytes, e.llv, e.n, e.nonspecials),
         lambda got: np.array_equal(got, itv_want)),
        ("bottomup", bottomup, lambda got: np.array_equal(got, pops)),
    ]


@pytest.mark.parametrize("idx", range(5))
def test_entry_keeps_current_device(idx):
    e = oracle_esa("at1MB")
    name, call, check = _calls(e)[idx]
    _set_device(0)
    got = call()
    assert _get_device() == 0, name
    assert check(got), name


@pytest.mark.skipif(G.device_count() < 2, reason="needs >= 2 visible GPUs")
@pytest.mark.parametrize("idx", range(5))
def test_entry_on_device_1(idx):
    """Called with device 1 current: the work runs there and device 1 is
    still current on return."""
    e = oracle_esa("at1MB")
    name, call, check = _calls(e)[idx]
    _set_device(1)
    try:
        got = call()
        assert _get_device() == 1, name
        assert check(got), name
    finally:
        _set_device(0)

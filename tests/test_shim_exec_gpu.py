"""Execution test of the reference-side binding (integration/esa_linsmax.c).

integration/exec_test/_build/shim_exec is the shim compiled against the
reference's headers and linked with libgtsmax_hip.so plus test doubles of
the gt reader/error/allocator functions (integration/exec_test/gt_stubs.c;
built in the container by __graft_entry__.build(), which has the reference
headers).  Its output function has the GtProcessmaxpairs type of the repfind
runner (src/match/esa-maxpairs.h:38-43, src/tools/gt_repfind.c:49-84) and
records every (len, pos1, pos2) call in order.  Expected, from the oracle:
  - smax: every occurrence pair of every interval, intervals in ascending lb,
    pairs in occurrence-row order (a outer, b inner) -- the order
    smax_shim_interval hands them to the runner;
  - maxpairs: orc_maxpairs, the reference's emission order (its own golden
    testdata/repfind-8-Atinsert.txt pins it, tests/test_oracle.py);
mapped 8-byte .suf and -scan with the 4-byte .suf of -suftabuint
(src/match/esa-map.c:362-381), 1 and 2 shards.
"""
import os
import subprocess

import numpy as np
import pytest

import oracle_lib as O
from conftest import GOLDEN, oracle_esa

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM_EXEC = os.path.join(ROOT, "integration", "exec_test", "_build", "shim_exec")


def _run(index, minlen, mode, *extra):
    if not os.path.isfile(SHIM_EXEC):
        pytest.fail("integration/exec_test/_build/shim_exec missing: run __graft_entry__.build() "
                    "in the container that holds the reference headers")
    r = subprocess.run([SHIM_EXEC, index, str(minlen), mode] + [str(x) for x in extra],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    rows = [tuple(int(v) for v in line.split()) for line in r.stdout.splitlines()]
    return np.array(rows, dtype=np.uint64).reshape(-1, 3)


def _smax_pairs(e, minlen):
    iv = O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, minlen)
    return np.array(O.smax_pairs(iv, e.suftab), dtype=np.uint64).reshape(-1, 3)


@pytest.fixture(scope="module")
def indexes(tmp_path_factory):
    d = tmp_path_factory.mktemp("idx")
    out = {}
    for name in ("Atinsert.fna", "at1MB"):
        for w in (8, 4):
            idx = str(d / ("%s_%d" % (name.split(".")[0], w)))
            O.index_fasta(os.path.join(GOLDEN, name), idx, suftab_bytes=w)
            out[(name, w)] = idx
    return out


@pytest.mark.parametrize("name,minlen", [("Atinsert.fna", 8), ("at1MB", 20), ("at1MB", 300)])
@pytest.mark.parametrize("how", [("mapped", 8, 1), ("mapped", 8, 2), ("scan", 4, 1),
                                 ("scan", 8, 1)])
def test_smax_pairs_through_the_shim(indexes, name, minlen, how):
    mode, width, gpus = how
    e = oracle_esa(name)
    want = _smax_pairs(e, minlen)
    extra = (["-scan"] if mode == "scan" else []) + [gpus]
    got = _run(indexes[(name, width)], minlen, "smax", *extra)
    assert len(want) > 0
    assert np.array_equal(got, want), (len(got), len(want))


@pytest.mark.parametrize("name,minlen", [("Atinsert.fna", 8), ("at1MB", 20)])
@pytest.mark.parametrize("mode,width", [("mapped", 8), ("scan", 4)])
def test_maxpairs_through_the_shim(indexes, name, minlen, mode, width):
    e = oracle_esa(name)
    want = O.maxpairs(e, minlen)
    extra = ["-scan"] if mode == "scan" else []
    got = _run(indexes[(name, width)], minlen, "maxpairs", *extra)
    assert len(want) > 0
    assert np.array_equal(got, want), (len(got), len(want))


@pytest.mark.parametrize("name", ["Atinsert.fna", "at1MB"])
def test_esa_bottomup_gpu_drives_a_gt_visitor(tmp_path, name):
    """gt_esa_bottomup_gpu (the shim's replacement of gt_esa_bottomup,
    src/match/esa-bottomup.h:31-33) drives a GtESAVisitor through the
    reference's gt_esa_visitor_* calls (a recording double): every call,
    its GtESAVisitorInfo objects (stack-slot identity, creation order) and
    their deletion equal the reference traversal's
    (orc_bottomup_events_slots, esa-bottomup.c:20-273)."""
    if not os.path.isfile(SHIM_EXEC):
        pytest.fail("integration/exec_test/_build/shim_exec missing")
    idx = str(tmp_path / "idx")
    O.index_fasta(os.path.join(GOLDEN, name), idx)
    r = subprocess.run([SHIM_EXEC, idx, "0", "bottomup"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr
    calls, deleted = [], []
    for line in r.stdout.splitlines():
        f = line.split()
        if f[0] == "D":
            deleted.append(int(f[1]))
        else:
            calls.append([int(x) for x in f])
    got = np.array(calls, dtype=np.uint64).reshape(-1, 9)
    e = oracle_esa(name)
    ev, sl, nslots = O.bottomup_events_slots(e)
    none = np.uint64(2 ** 64 - 1)
    ids = np.where(sl == none, np.uint64(0), sl + np.uint64(1))
    ids[ev[:, 0] != 1, 1] = 0
    assert np.array_equal(got[:, :7], ev)
    assert np.array_equal(got[:, 7:], ids)
    assert deleted == list(range(1, nslots + 1))

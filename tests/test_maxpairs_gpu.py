"""GPU parity for maximal pairs (`gt repfind -l N`) and the
on-device seqnum/relpos mapping (F4), through the C-ABI.

Pinned to the reference's own golden `testdata/repfind-8-Atinsert.txt`
(`gt repfind -l 8` on Atinsert, 452 lines) line for line, and to the
oracle's restatement of the bottom-up maxpairs traversal
(`orc_maxpairs`, src/match/esa-bottomup-maxpairs.inc:136-264) on fixtures and
seeded texts with specials and .llv values.  The host entry points and
`emit_ordered` emit in the reference's order, each call's (pos1, pos2) in
the reference's argument order: compared pair by pair (exactly on the
fixtures; elsewhere as (len, min pos, max pos), the swap
gt_simpleexactselfmatchoutput makes); the row-order device pass
(`plan.emit`) is compared as a set.
"""
import os

import numpy as np
import pytest

import genometools_smax_amd as G
import oracle_lib as O
from conftest import GOLDEN, oracle_esa

pytestmark = pytest.mark.gpu


def _norm(p):
    p = np.asarray(p, dtype=np.uint64).reshape(-1, 3)
    lo = np.minimum(p[:, 1], p[:, 2])
    hi = np.maximum(p[:, 1], p[:, 2])
    q = np.stack([p[:, 0], lo, hi], axis=1)
    return q[np.lexsort((q[:, 2], q[:, 1], q[:, 0]))]


def _gpu(e, minlen, suf_dtype=np.uint64):
    return G.enumerate_maxpairs(e.lcpbytes, e.llv, e.bwt, e.suftab.astype(suf_dtype), e.n,
                                e.nonspecials, minlen)


def test_atinsert_matches_reference_golden():
    e = oracle_esa("Atinsert.fna")
    got = _gpu(e, 8)
    lines = [" ".join(ln.split()) for ln in O.format_pairs(got, e.separators)]
    with open(os.path.join(GOLDEN, "repfind-8-Atinsert.txt")) as fh:
        want = [" ".join(ln.split()) for ln in fh if ln.strip()]
    assert len(lines) == 452
    assert lines == want                  # the reference's own order, line by line


@pytest.mark.parametrize("minlen", [4, 8, 12, 20, 40])
def test_atinsert_pair_set(minlen):
    e = oracle_esa("Atinsert.fna")
    got = _gpu(e, minlen)
    # the reference's calls exactly: order and pos1/pos2 argument order
    assert np.array_equal(got, O.maxpairs(e, minlen))


@pytest.mark.parametrize("minlen", [20, 50, 255, 300])
def test_at1mb_pair_set(minlen):
    e = oracle_esa("at1MB")
    got = _gpu(e, minlen)
    assert np.array_equal(got, O.maxpairs(e, minlen))
    if minlen == 20:
        assert len(O.format_pairs(got, e.separators)) == 4507


def test_suftab_4_bytes():
    e = oracle_esa("at1MB")
    assert np.array_equal(_gpu(e, 20, np.uint32), _gpu(e, 20))


def _repetitive(rng, n, pspecial):
    t = rng.integers(0, 4, n, dtype=np.uint8)
    fams = [rng.integers(0, 4, int(rng.integers(40, 600)), dtype=np.uint8) for _ in range(5)]
    for _ in range(n // 2000):
        f = fams[int(rng.integers(0, len(fams)))]
        at = int(rng.integers(0, n - len(f)))
        cp = f.copy()
        mut = rng.random(len(cp)) < 0.02
        cp[mut] = rng.integers(0, 4, int(mut.sum()), dtype=np.uint8)
        t[at:at + len(cp)] = cp
    sp = rng.random(n) < pspecial
    t[sp] = rng.choice(np.array([254, 255], dtype=np.uint8), int(sp.sum()))
    return t


@pytest.mark.parametrize("seed", range(4))
def test_random_repetitive(seed):
    rng = np.random.default_rng(300 + seed)
    t = _repetitive(rng, int(rng.integers(20000, 80000)), [0.0, 0.001, 0.01, 0.05][seed])
    e = O.Esa(t)
    for minlen in (12, 30, 256):
        assert np.array_equal(_gpu(e, minlen), O.maxpairs(e, minlen)), minlen


@pytest.mark.parametrize("rank_max", ["0", "1000000000"])
def test_ordered_pass_rank_and_radix_paths(monkeypatch, rank_max):
    # emit_ordered sorts a small pass (T <= GT_MP_RANK_MAX, 16384 by default)
    # by rank counting and a larger one by stable LSD radix passes; both must
    # give the reference's calls exactly, forced either way here
    monkeypatch.setenv("GT_MP_RANK_MAX", rank_max)
    e = oracle_esa("at1MB")
    for minlen in (8, 20):
        assert np.array_equal(_gpu(e, minlen), O.maxpairs(e, minlen)), minlen
    rng = np.random.default_rng(303)
    e = O.Esa(_repetitive(rng, 60000, 0.01))
    for minlen in (12, 30):
        assert np.array_equal(_gpu(e, minlen), O.maxpairs(e, minlen)), minlen


def test_count_pass_separate_scan_path(monkeypatch):
    # GT_MP_LOOKBACK=0: the count pass as count, scan and write kernels (the
    # default fuses each pair with a decoupled look-back)
    monkeypatch.setenv("GT_MP_LOOKBACK", "0")
    e = oracle_esa("at1MB")
    for minlen in (8, 20, 300):
        assert np.array_equal(_gpu(e, minlen), O.maxpairs(e, minlen)), minlen
    e = O.Esa(_repetitive(np.random.default_rng(304), 50000, 0.01))
    assert np.array_equal(_gpu(e, 12), O.maxpairs(e, 12))


def test_count_passes_past_the_status_tag_wrap():
    # the look-back status words carry the pass number mod 65535: 70,000
    # count passes on one plan (the tag wraps once) keep the same list,
    # offsets and total
    import torch
    e = oracle_esa("at1MB")
    d = G.DeviceEsa(e.text, keep_suftab=True)
    p = d.maxpairs_plan(20)
    want = O.maxpairs(e, 20)
    out = torch.empty(3 * len(want), dtype=torch.int64, device="cuda")
    for k in range(70000):
        p.count()
        if k in (0, 65534, 65535, 65536, 69999):
            assert p.total() == len(want), k
            p.emit_ordered(out.data_ptr(), len(want))
            assert np.array_equal(out.cpu().numpy().view(np.uint64).reshape(-1, 3), want), k
    p.close()
    d.release()


def test_long_lcp_values():
    # an exact 1200-symbol duplication: pairs of length >= 255 need the .llv
    rng = np.random.default_rng(9)
    a = rng.integers(0, 4, 1200, dtype=np.uint8)
    t = np.concatenate([rng.integers(0, 4, 5000, dtype=np.uint8), a, np.array([255], np.uint8),
                        rng.integers(0, 4, 3000, dtype=np.uint8), a, np.array([254], np.uint8), a])
    e = O.Esa(t)
    assert len(e.llv) > 0
    for minlen in (100, 255, 256, 1000, 1200, 1201):
        assert np.array_equal(_gpu(e, minlen), O.maxpairs(e, minlen)), minlen


@pytest.mark.parametrize("seed", range(4))
def test_small_edge_texts(seed):
    rng = np.random.default_rng(40 + seed)
    for _ in range(15):
        n = int(rng.integers(1, 200))
        t = rng.integers(0, int(rng.integers(1, 5)), n, dtype=np.uint8)
        if rng.random() < 0.5:
            t[rng.random(n) < 0.1] = 254
        e = O.Esa(t)
        for minlen in (1, 2, 5):
            assert np.array_equal(_gpu(e, minlen), O.maxpairs(e, minlen))


def test_device_resident_plan_and_seqpos_map():
    import torch
    e = oracle_esa("at1MB")
    d = G.DeviceEsa(e.text, keep_suftab=True)
    p = d.maxpairs_plan(20)
    p.count()
    total = p.total()
    out = torch.empty(3 * total, dtype=torch.int64, device="cuda")
    p.emit(out.data_ptr(), total)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint64).reshape(-1, 3)
    assert np.array_equal(_norm(got), _norm(O.maxpairs(e, 20)))
    ordered = torch.empty(3 * total, dtype=torch.int64, device="cuda")
    p.emit_ordered(ordered.data_ptr(), total)
    assert np.array_equal(ordered.cpu().numpy().view(np.uint64).reshape(-1, 3),
                          O.maxpairs(e, 20))
    # F4: seqnum / relpos on the device == the oracle's formatter
    sep = torch.from_numpy(e.separators.view(np.int64)).cuda()
    mapped = torch.empty(5 * total, dtype=torch.int64, device="cuda")
    G.seqpos_map_dev(sep.data_ptr(), len(e.separators), out.data_ptr(), total, mapped.data_ptr())
    torch.cuda.synchronize()
    m = mapped.cpu().numpy().view(np.uint64).reshape(-1, 5)
    lines = ["%d %d %d F %d %d %d\n" % (r[0], r[1], r[2], r[0], r[3], r[4]) for r in m]
    assert sorted(lines) == sorted(O.format_pairs(got, e.separators))
    p.close()
    d.release()


def test_errors_are_reported():
    e = oracle_esa("Atinsert.fna")
    with pytest.raises(G.SmaxError):
        G.enumerate_maxpairs(e.lcpbytes, e.llv, e.bwt, e.suftab, e.n, e.n + 5, 8)
    with pytest.raises(G.SmaxError):
        G.enumerate_maxpairs(e.lcpbytes, e.llv, e.bwt, e.suftab, e.n, e.nonspecials, 0)


class _TablesEsa:
    """Oracle view (exact LCP, suftab, text) of GPU-built tables."""

    def __init__(self, text, d):
        self.text = np.ascontiguousarray(text, dtype=np.uint8)
        self.n = len(text)
        self.nonspecials = int(self.n - np.count_nonzero(text >= 254))
        self.lcp = d["lcptab"].astype(np.uint64)
        if len(d["llvtab"]):
            self.lcp[d["llvtab"][:, 0].astype(np.int64)] = d["llvtab"][:, 1]
        self.suftab = d["suftab"].astype(np.uint64)


@pytest.mark.parametrize("runlen", [100_000, 1_000_000])
def test_homopolymer_block_costs_its_output(runlen):
    # one block of ~runlen rows whose suffixes share their left symbol: the
    # walk skips runs of j's left symbol (linear, not quadratic, in the block)
    import time
    rng = np.random.default_rng(runlen)
    text = np.concatenate([rng.integers(0, 4, 200_000, dtype=np.uint8),
                           np.zeros(runlen, dtype=np.uint8),
                           rng.integers(0, 4, 200_000, dtype=np.uint8)])
    esa = G.DeviceEsa(text, device=0, keep_suftab=True)
    d = esa.download(suftab=True)
    esa.release()
    N = len(text)
    t0 = time.perf_counter()
    got = G.enumerate_maxpairs(d["lcptab"], d["llvtab"], d["bwttab"], d["suftab"], N, N, 20)
    dt = time.perf_counter() - t0
    want = O.maxpairs(_TablesEsa(text, d), 20)
    assert len(want) > runlen // 2
    assert np.array_equal(got, want)
    assert dt < 20.0, dt


def test_lcp_255_without_llv_is_an_error():
    e = oracle_esa("at1MB")
    llv = e.llv[1:]                      # drop one entry: its 255 byte is orphaned
    with pytest.raises(G.SmaxError, match="255"):
        G.enumerate_maxpairs(e.lcpbytes, llv, e.bwt, e.suftab, e.n, e.nonspecials, 20)


def test_smax_lines_edge_values_and_chunks():
    # F4 formatter on its own: positions up to ~2^40, separators spread
    # over them, a 2900-occurrence record (4.2 M pairs: more than one 2^22
    # chunk), 0-length-digit edges; against the oracle's restatement of
    # gt_querymatch_output line by line
    rng = np.random.default_rng(77)
    sep = np.unique(rng.integers(1, 1 << 40, 5000, dtype=np.uint64))
    sep = np.concatenate([np.array([0, 9, 10, 99, 100], dtype=np.uint64), sep])
    sep = np.unique(sep)
    widths = [2900] + [int(w) for w in rng.integers(2, 6, 300)]
    occ, recs, at = [], [], 0
    for k, w in enumerate(widths):
        pos = rng.integers(0, 1 << 40, w, dtype=np.uint64)
        pos = pos[~np.isin(pos, sep)]
        if len(pos) < 2:
            continue
        occ.append(pos)
        recs.append((at, int(rng.integers(1, 1 << 31)), len(pos)))
        at += len(pos)
    occ = np.concatenate(occ)
    rec = np.array(recs, dtype=G.RECORD_DTYPE)
    text = G.format_smax_lines(rec, occ, sep)
    small = [(int(r["lcp"]), int(a), int(b))
             for r in rec[1:] for i, a in enumerate(occ[r["lb"]:r["lb"] + r["width"]])
             for b in occ[r["lb"] + i + 1:r["lb"] + r["width"]]]
    lines = text.decode().splitlines(keepends=True)
    w0 = int(rec[0]["width"])
    n0 = w0 * (w0 - 1) // 2
    assert len(lines) == n0 + len(small)
    assert lines[n0:] == O.format_pairs(small, sep)
    # the big record: every 997th pair plus the chunk seam
    o0 = occ[:w0]
    pairs0 = [(a, b) for a in range(w0) for b in range(a + 1, w0)]
    pick = sorted(set(list(range(0, n0, 997)) + [(1 << 22) - 1, 1 << 22, n0 - 1]))
    want = O.format_pairs([(int(rec[0]["lcp"]), int(o0[pairs0[k][0]]), int(o0[pairs0[k][1]]))
                           for k in pick], sep)
    assert [lines[k] for k in pick] == want


def test_maxpairs_lines_dev_equal_oracle_lines():
    import torch
    e = oracle_esa("at1MB")
    got = _gpu(e, 20)
    pairs = torch.from_numpy(got.view(np.int64).reshape(-1)).cuda()
    sep = torch.from_numpy(np.ascontiguousarray(e.separators).view(np.int64)).cuda()
    text = G.repfind_pairs_lines_dev(pairs.data_ptr(), len(got), sep.data_ptr(), len(e.separators))
    assert text.decode().splitlines(keepends=True) == O.format_pairs(O.maxpairs(e, 20), e.separators)


def test_python_repfind_smax_lines():
    e = oracle_esa("Atinsert.fna")
    itv = O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, 8)
    got = G.repfind_smax_lines(itv, e.suftab, e.separators)
    want = [w.rstrip("\n") for w in O.format_pairs(O.smax_pairs(itv, e.suftab), e.separators)]
    assert len(got) == 205 and got == want

"""Pins the CPU oracle to the reference's own fixtures (no GPU needed).

Parity anchors (the reference is unbuildable here -- see DESIGN.md):
  * testdata/repfind-8-Atinsert.txt: `gt repfind -l 8` on Atinsert, compared
    in gt_idxsearch_include.rb:144-154 with diff -w.  The oracle's ESA +
    maxpairs restatement must reproduce it line for line, in order.
  * testdata/prj-files/*.prj: .prj statistics of gt suffixerator runs.
  * SURVEY.md §8(c) verified counts from the reference build (Atinsert l=8:
    114 smax / 263 occurrences / 205 pairs; at1MB l=20: n=772,376,
    N=753,453, 2,317 llv entries, max lcp 517, 38,153 local maxima,
    884 / 1,771 / 890, 4,507 repfind lines).
"""
import os

import numpy as np
import pytest

import oracle_lib as O
from conftest import GOLDEN, oracle_esa


def _norm(lines):
    return [" ".join(l.split()) for l in lines if l.strip() and not l.startswith("#")]


def test_maxpairs_reproduces_repfind_golden():
    e = oracle_esa("Atinsert.fna")
    lines = O.format_pairs(O.maxpairs(e, 8), e.separators)
    with open(os.path.join(GOLDEN, "repfind-8-Atinsert.txt")) as fh:
        gold = _norm(fh)
    assert _norm(lines) == gold
    assert len(gold) == 452


def test_atinsert_smax_known_answer():
    e = oracle_esa("Atinsert.fna")
    assert (e.n, e.nonspecials) == (11817, 8867)
    a = O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, 8)
    assert len(a) == 114
    assert int((a[:, 2] - a[:, 1] + 1).sum()) == 263
    pairs = O.format_pairs(O.smax_pairs(a, e.suftab), e.separators)
    assert len(pairs) == 205
    with open(os.path.join(GOLDEN, "repfind-8-Atinsert.txt")) as fh:
        gold = set(_norm(fh))
    assert set(_norm(pairs)) <= gold


def _local_maxima(lcp, N, minlen):
    L = lcp[: N + 1].astype(np.int64).copy()
    L[0] = 0
    L[N] = 0
    cnt = 0
    k = 1
    while k <= N - 1:
        if L[k] > L[k - 1] and L[k] >= minlen:
            j = k
            while j + 1 <= N - 1 and L[j + 1] == L[k]:
                j += 1
            nxt = L[j + 1] if j + 1 <= N - 1 else 0
            if nxt < L[k]:
                cnt += 1
            k = j + 1
        else:
            k += 1
    return cnt


def test_at1mb_known_answer():
    e = oracle_esa("at1MB")
    assert (e.n, e.nonspecials) == (772376, 753453)
    assert len(e.llv) == 2317
    assert int(e.lcp.max()) == 517
    assert _local_maxima(e.lcp, e.nonspecials, 20) == 38153
    a = O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, 20)
    assert len(a) == 884
    assert int((a[:, 2] - a[:, 1] + 1).sum()) == 1771
    mp = O.format_pairs(O.maxpairs(e, 20), e.separators)
    assert len(mp) == 4507
    sp = O.format_pairs(O.smax_pairs(a, e.suftab), e.separators)
    assert len(sp) == 890
    assert set(_norm(sp)) <= set(_norm(mp))


@pytest.mark.parametrize("minlen", [1, 4, 8, 12, 20])
def test_linsmax_equals_bottomup_atinsert(minlen):
    e = oracle_esa("Atinsert.fna")
    a = O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, minlen)
    b = O.bottomup_smax(e, minlen)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("minlen", [10, 50, 255, 300])
def test_linsmax_equals_bottomup_at1mb(minlen):
    e = oracle_esa("at1MB")
    a = O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, minlen)
    b = O.bottomup_smax(e, minlen)
    assert np.array_equal(a, b)



@pytest.mark.parametrize("threads", [2, 3, 7, 64])
def test_linsmax_all_core_equals_single(threads):
    """orc_linsmax_mt (bench's all-core CPU figure) == orc_linsmax, incl. ranges
    that cut plateaus and .llv runs (tandem text: long plateaus, many .llv)."""
    for name, minlen in (("at1MB", 20), ("at1MB", 256), ("Atinsert.fna", 1)):
        e = oracle_esa(name)
        a = O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, minlen)
        b = O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, minlen, threads=threads)
        assert np.array_equal(a, b)
    t = np.tile(np.array([0, 1, 2, 0, 3], np.uint8), 400)
    e = O.Esa(t)
    for minlen in (1, 300):
        a = O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, minlen)
        b = O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, minlen, threads=threads)
        assert np.array_equal(a, b)

def _random_text(rng, n, sigma=4, pspecial=0.02):
    t = rng.integers(0, sigma, n, dtype=np.uint8)
    sp = rng.random(n) < pspecial
    t[sp] = rng.choice(np.array([254, 255], dtype=np.uint8), sp.sum())
    return t


@pytest.mark.parametrize("seed", range(12))
def test_three_derivations_agree_random(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(2, 220))
    sigma = int(rng.integers(1, 5))
    t = _random_text(rng, n, sigma, pspecial=float(rng.choice([0.0, 0.03, 0.2])))
    if seed % 3 == 0:   # tandem repeats give long plateaus / nested intervals
        unit = rng.integers(0, sigma, int(rng.integers(1, 6)), dtype=np.uint8)
        t = np.tile(unit, n // len(unit) + 1)[:n].copy()
    e = O.Esa(t)
    for minlen in (1, 2, 3, 5):
        a = O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, minlen)
        b = O.bottomup_smax(e, minlen)
        assert np.array_equal(a, b)
        brute = O.brute_smax(t, minlen)
        esa_sets = sorted((int(l), tuple(sorted(int(e.suftab[k]) for k in range(lb, rb + 1))))
                          for l, lb, rb in a)
        assert esa_sets == sorted(brute)


def test_special_example_from_survey():
    # >t ACACNACAC  >u ACAC : smax ACAC with 3 occurrences
    t = np.array([0, 1, 0, 1, 254, 0, 1, 0, 1, 255, 0, 1, 0, 1], dtype=np.uint8)
    e = O.Esa(t)
    assert (e.n, e.nonspecials) == (14, 12)
    assert list(e.suftab[:3]) == [0, 5, 10]
    assert list(e.bwt[:3]) == [254, 254, 255]
    a = O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, 4)
    assert a.tolist() == [[4, 0, 2]]


def _prj(path):
    out = {}
    with open(path) as fh:
        for line in fh:
            if "=" in line and not line.startswith("dbfile"):
                k, v = line.strip().split("=")
                out[k] = v
    return out


@pytest.mark.parametrize("fasta,prj", [
    (["Random-Small.fna"], "Random-Small.prj"),
    (["Random.fna"], "Random.prj"),
    (["TTT-small.fna"], "TTT-small.prj"),
    (["Atinsert.fna", "Random.fna"], "Atinsert+Random.prj"),
])
def test_prj_statistics_match_reference(tmp_path, fasta, prj):
    cat = tmp_path / "in.fna"
    with open(cat, "wb") as out:
        for f in fasta:
            with open(os.path.join(GOLDEN, f), "rb") as fh:
                data = fh.read()
            out.write(data if data.endswith(b"\n") else data + b"\n")
    idx = str(tmp_path / "idx")
    O.index_fasta(str(cat), idx)
    mine, ref = _prj(idx + ".prj"), _prj(os.path.join(GOLDEN, "prj", prj))
    for key in ("totallength", "specialcharacters", "specialranges", "realspecialranges",
                "lengthofspecialprefix", "lengthofspecialsuffix", "numofsequences",
                "largelcpvalues", "readmode"):
        assert mine[key] == ref[key], key


def test_index_files_layout(tmp_path):
    idx = str(tmp_path / "at")
    O.index_fasta(os.path.join(GOLDEN, "Atinsert.fna"), idx)
    e = oracle_esa("Atinsert.fna")
    n = e.n
    assert os.path.getsize(idx + ".suf") == 8 * (n + 1)
    assert os.path.getsize(idx + ".lcp") == n + 1
    assert os.path.getsize(idx + ".bwt") == n + 1
    assert os.path.getsize(idx + ".llv") == 0
    assert np.array_equal(np.fromfile(idx + ".suf", dtype=np.uint64), e.suftab)
    O.index_fasta(os.path.join(GOLDEN, "Atinsert.fna"), idx + "4", suftab_bytes=4)
    assert np.array_equal(np.fromfile(idx + "4.suf", dtype=np.uint32).astype(np.uint64), e.suftab)


@pytest.mark.parametrize("name", ["Atinsert.fna", "at1MB"])
def test_bottomup_event_stream_shape(name):
    # gt_esa_bottomup restatement (F3 checker): one leaf edge per suffix,
    # one branching edge per popped interval, intervals in pop order
    # (rb ascending, then depth descending), exactly one firstsucc root edge
    e = oracle_esa(name)
    ev = O.bottomup_events(e)
    kinds = ev[:, 0]
    assert int((kinds == 0).sum()) == e.nonspecials
    assert int((kinds == 1).sum()) == int((kinds == 2).sum())
    itv = ev[kinds == 2]
    order = np.lexsort((-itv[:, 2].astype(np.int64), itv[:, 4]))
    assert np.array_equal(order, np.arange(len(itv)))
    root = ev[(kinds != 2) & (ev[:, 2] == 0)]
    assert int(root[:, 1].sum()) == 1 and root[0, 1] == 1
    # the smax intervals are exactly the lcp-intervals without a branching
    # child that pass the diversity test: a subset of the intervals
    sm = O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, 8)
    allitv = set(map(tuple, itv[:, 2:5].tolist()))
    assert set(map(tuple, sm.tolist())) <= allitv


def _lb_lines(ev):
    """L/B records of an event stream as the lcpitvs visitor prints them
    (srb and the lcp-interval events are not printed)."""
    ev = ev[ev[:, 0] != 2].copy()
    ev[:, 6] = 0
    return ev


@pytest.mark.parametrize("name", ["Reads2.fna", "Atinsert.fna", "Random.fna", "TTT-small.fna",
                                  "at1MB"])
def test_dfs_lines_equal_bottomup_lines(name):
    # the reference's own lcp-interval test (testsuite/gt_suffixerator_include.rb:
    # 597-603): `gt dev sfxmap -enumlcpitvtreeBU` == `-enumlcpitvtree` on
    # Reads2.fna; here the restatements of both traversals (esa-bottomup.c,
    # esa-dfs.c + esa-lcpintervals.c) on it and the other fixtures
    e = oracle_esa(name)
    dfs = O.dfs_events(e)
    assert len(dfs) > 0
    assert np.array_equal(dfs, _lb_lines(O.bottomup_events(e)))


@pytest.mark.parametrize("seed", range(4))
def test_dfs_lines_equal_bottomup_lines_random(seed):
    rng = np.random.default_rng(900 + seed)
    for _ in range(30):
        n = int(rng.integers(1, 3000))
        t = rng.integers(0, int(rng.integers(1, 5)), n, dtype=np.uint8)
        if seed % 2:
            t[rng.random(n) < 0.02] = rng.choice(np.array([254, 255], np.uint8))
        e = O.Esa(t)
        assert np.array_equal(O.dfs_events(e), _lb_lines(O.bottomup_events(e)))


def test_prj_longest_is_row_of_suffix_0(tmp_path):
    """longest= (src/match/sfx-outprj.c:70-73) is the row holding suffix 0;
    esa-map.c:384-387 refuses a .suf load without it."""
    idx = str(tmp_path / "at")
    O.index_fasta(os.path.join(GOLDEN, "Atinsert.fna"), idx)
    e = oracle_esa("Atinsert.fna")
    assert int(_prj(idx + ".prj")["longest"]) == int(np.flatnonzero(e.suftab == 0)[0])


def _bottomup_tables_cases():
    for name, minlens in (("Atinsert.fna", (1, 8, 20)), ("at1MB", (10, 20, 255, 300, 517))):
        yield name, minlens


@pytest.mark.parametrize("name,minlens", list(_bottomup_tables_cases()))
def test_bottomup_over_tables_equals_linsmax(name, minlens):
    """orc_bottomup_smax_tables (the stack walk over .lcp/.llv/.bwt as the
    sequential reader hands them out; bench.py's reference-algorithm CPU
    anchor) == orc_linsmax over all rows."""
    e = oracle_esa(name)
    for minlen in minlens:
        a = O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, minlen)
        b = O.bottomup_smax_tables(e.lcpbytes, e.llv, e.bwt, e.nonspecials, minlen)
        assert np.array_equal(a, b), (name, minlen)


@pytest.mark.parametrize("seed", range(6))
def test_bottomup_over_tables_random(seed):
    rng = np.random.default_rng(100 + seed)
    t = _random_text(rng, int(rng.integers(2, 400)), int(rng.integers(1, 5)), 0.03)
    if seed % 2:
        t = np.tile(t[:5], 80)
    e = O.Esa(t)
    for minlen in (1, 2, 5, 300):
        a = O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, minlen)
        b = O.bottomup_smax_tables(e.lcpbytes, e.llv, e.bwt, e.nonspecials, minlen)
        assert np.array_equal(a, b)


def _intervals_from_events(ev):
    """(lcp, lb, rb, fatherlcp, fatherlb) of every popped interval: each
    visit_lcp_interval event is followed by its branching edge to the father."""
    out = []
    for k in np.flatnonzero(ev[:, 0] == 2):
        l, lb, rb = ev[k, 2:5]
        assert ev[k + 1, 0] == 1 and tuple(ev[k + 1, 4:7]) == (l, lb, rb)
        out.append((l, lb, rb, ev[k + 1, 2], ev[k + 1, 3]))
    return np.array(out, dtype=np.uint64).reshape(-1, 5)


@pytest.mark.parametrize("name", ["Atinsert.fna", "at1MB", "Reads2.fna", "TTT-small.fna"])
def test_lcp_intervals_equal_bottomup_events(name):
    """orc_lcp_intervals (F3's checker past 2^32 rows: tables only, no
    suffix array) == the intervals and fathers of orc_bottomup_events."""
    e = oracle_esa(name)
    want = _intervals_from_events(O.bottomup_events(e))
    got = O.lcp_intervals(e.lcpbytes, e.llv, e.nonspecials, cap=e.nonspecials + 1)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("name,minlen", [("Atinsert.fna", 8), ("Atinsert.fna", 14),
                                         ("at1MB", 20), ("at1MB", 300)])
def test_maxpairs_blocks_equal_maxpairs(name, minlen):
    """orc_maxpairs_blocks (maximal pairs by definition, per block; F2's
    checker past 2^32 rows) == orc_maxpairs as a set."""
    e = oracle_esa(name)
    want = O.maxpairs(e, minlen)
    got = O.maxpairs_blocks(e.lcpbytes, e.llv, e.bwt, e.suftab, e.nonspecials, minlen,
                            cap=len(want) + 16)
    def key(a):
        a = np.column_stack([a[:, 0], np.sort(a[:, 1:], axis=1)])
        return a[np.lexsort(a.T[::-1])]
    assert len(want) > 0
    assert np.array_equal(key(got), key(want))


NONE = np.uint64(2 ** 64 - 1)


def _leafcount_visit(ev, sl):
    """A visitor with per-node state (the leaves below each interval), run
    over an event stream with its stack slots the way gt_esa_bottomup hands
    GtESAVisitorInfo objects to a visitor: returns the intervals whose count
    is not rb - lb + 1 (none, if the slot model is the reference's)."""
    state, bad = {}, []
    for (t, f, a, b, c, d, e), (s0, s1) in zip(ev.tolist(), sl.tolist()):
        if t == 0:
            state[s0] = 1 if f else state[s0] + 1
        elif t == 1:
            if s1 == int(NONE):            # father pushed into its first child's slot
                assert f == 1 and b == d   # same lb: the child's state carries over
            elif f:
                state[s0] = state[s1]
            else:
                state[s0] += state[s1]
        elif state[s0] != c - b + 1:
            bad.append((a, b, c))
    return bad


@pytest.mark.parametrize("name", ["Atinsert.fna", "at1MB", "Reads2.fna", "TTT-small.fna"])
def test_event_slots_model_visitor_info(name):
    """orc_bottomup_events_slots: same events as orc_bottomup_events, and the
    stack slots (the reference's GtESAVisitorInfo, esa-bottomup.c:20-110)
    carry a per-node leaf count correctly -- the model F3's info visitor
    (gt_esa_bottomup_info_hip) is checked against."""
    e = oracle_esa(name)
    ev, sl, nslots = O.bottomup_events_slots(e)
    assert np.array_equal(ev, O.bottomup_events(e))
    assert nslots % 32 == 0 and nslots > 0
    used = sl[sl != NONE]
    assert used.max() < nslots
    assert _leafcount_visit(ev, sl) == []


@pytest.mark.parametrize("seed", range(6))
def test_event_slots_random(seed):
    rng = np.random.default_rng(700 + seed)
    t = _random_text(rng, int(rng.integers(2, 3000)), int(rng.integers(1, 5)), 0.02)
    if seed % 2:                           # a run of the largest symbol before a smaller
        run = np.full(int(rng.integers(40, 200)), 3, np.uint8)   # one: LCPs rise row by row,
        t = np.concatenate([t[:50], run, np.zeros(1, np.uint8), t[50:100]])   # > 32 slots
    e = O.Esa(t)
    ev, sl, nslots = O.bottomup_events_slots(e)
    assert _leafcount_visit(ev, sl) == []
    if seed % 2:
        assert nslots > 32


# ------------------------------------------------- spmitv (F3 visitor golden)
# `gt dev sfxmap -spmitv` on an index of Reads2.fna (-suf -lcp) must print
# testdata/Reads2-spmitv.txt (testsuite/gt_suffixerator_include.rb:587-592):
# gt_esa_bottomup driving the spmitvs visitor (src/match/esa-spmitvs.c:25-69,
# src/match/esa_spmitvs_visitor.c:59-226).  This pins the oracle's bottom-up
# event stream -- leaf numbers, branching-edge depths and child bounds, every
# lcp-interval -- to a reference-produced file.

def _index_events(tmp_path, fasta):
    import genometools_smax_amd as G   # the host-side index reader (pure Python)
    idx = str(tmp_path / os.path.basename(fasta))
    O.index_fasta(os.path.join(GOLDEN, fasta), idx)
    ix = G.EsaIndex(idx)
    n, N = ix.totallength, ix.nonspecials
    lcp = np.asarray(ix.lcptab).astype(np.uint64)
    if len(ix.llvtab):
        lcp[np.asarray(ix.llvtab)[:, 0].astype(np.int64)] = np.asarray(ix.llvtab)[:, 1]

    class _E:
        pass
    e = _E()
    e.lcp, e.suftab, e.nonspecials = lcp, np.asarray(ix.suftab).astype(np.uint64), N
    sep_text = np.zeros(n, np.uint8)
    sep_text[ix.separators().astype(np.int64)] = 255      # the encseq's separators
    return ix, e, sep_text


def test_spmitv_reproduces_reads2_golden(tmp_path):
    ix, e, sep_text = _index_events(tmp_path, "Reads2.fna")
    lines = O.spmitv_lines(O.bottomup_events(e), sep_text, ix.nonspecials)
    with open(os.path.join(GOLDEN, "Reads2-spmitv.txt")) as fh:
        gold = fh.read().splitlines()
    assert len(gold) == 51
    assert lines == gold


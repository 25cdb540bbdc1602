"""GPU parity: the HIP smax path (through the C-ABI) against the CPU oracle.

Bit-exact comparison of the (lcp, lb, rb) interval lists, ascending lb, on
the reference's fixtures (Atinsert, at1MB), on seeded random/repetitive
texts (specials, long plateaus, .llv overflow values) and across shard
counts (the boundary stitch), at sizes the oracle finishes in seconds.
"""
import numpy as np
import pytest

import genometools_smax_amd as G
import oracle_lib as O
from conftest import oracle_esa

pytestmark = pytest.mark.gpu


def _gpu(e, minlen, shards=1):
    return G.enumerate_smax(e.lcpbytes, e.llv, e.bwt, e.n, e.nonspecials, minlen, shards)


def _cpu(e, minlen):
    return O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, minlen)


def test_device_present():
    assert G.device_count() >= 1


@pytest.mark.parametrize("minlen", [1, 2, 4, 8, 12, 20, 40])
def test_atinsert(minlen):
    e = oracle_esa("Atinsert.fna")
    got, want = _gpu(e, minlen), _cpu(e, minlen)
    assert np.array_equal(got, want), (len(got), len(want))


def test_atinsert_known_answer():
    e = oracle_esa("Atinsert.fna")
    got = _gpu(e, 8)
    assert len(got) == 114 and int((got[:, 2] - got[:, 1] + 1).sum()) == 263


@pytest.mark.parametrize("minlen", [1, 5, 10, 20, 50, 200, 255, 256, 300, 517, 518])
def test_at1mb(minlen):
    e = oracle_esa("at1MB")
    got, want = _gpu(e, minlen), _cpu(e, minlen)
    assert np.array_equal(got, want), (len(got), len(want))


@pytest.mark.parametrize("shards", [2, 3, 5, 8, 17])
def test_at1mb_sharded(shards):
    e = oracle_esa("at1MB")
    want = _cpu(e, 20)
    got = _gpu(e, 20, shards)
    assert np.array_equal(got, want)


def _repetitive_text(rng, n, pspecial):
    # random genome with inserted copies of a few families (long lcps -> .llv)
    t = rng.integers(0, 4, n, dtype=np.uint8)
    fams = [rng.integers(0, 4, int(rng.integers(50, 800)), dtype=np.uint8) for _ in range(6)]
    pos = 0
    while pos < n:
        f = fams[int(rng.integers(0, len(fams)))]
        at = int(rng.integers(0, n))
        L = min(len(f), n - at)
        cp = f[:L].copy()
        mut = rng.random(L) < 0.01
        cp[mut] = rng.integers(0, 4, int(mut.sum()), dtype=np.uint8)
        t[at:at + L] = cp
        pos += L * 3
    sp = rng.random(n) < pspecial
    t[sp] = rng.choice(np.array([254, 255], dtype=np.uint8), int(sp.sum()))
    return t


@pytest.mark.parametrize("seed", range(6))
def test_random_repetitive(seed):
    rng = np.random.default_rng(100 + seed)
    n = int(rng.integers(20000, 200000))
    t = _repetitive_text(rng, n, [0.0, 0.001, 0.02][seed % 3])
    e = O.Esa(t)
    for minlen in (3, 10, 20, 100, 300):
        want = _cpu(e, minlen)
        assert np.array_equal(_gpu(e, minlen), want), minlen
        assert np.array_equal(_gpu(e, minlen, 1 + seed), want), (minlen, seed)


@pytest.mark.parametrize("seed", range(8))
def test_small_edge_texts(seed):
    rng = np.random.default_rng(seed)
    for _ in range(20):
        n = int(rng.integers(1, 300))
        sigma = int(rng.integers(1, 5))
        t = rng.integers(0, sigma, n, dtype=np.uint8)
        if rng.random() < 0.5:
            sp = rng.random(n) < 0.1
            t[sp] = 254
        e = O.Esa(t)
        for minlen in (1, 2, 3):
            want = _cpu(e, minlen)
            for shards in (1, 2, 4):
                assert np.array_equal(_gpu(e, minlen, shards), want)


def test_tandem_runs_cross_tiles():
    # homopolymer / short-period tandem repeats: plateaus and lcp ramps that
    # straddle 16384-row tiles and shard boundaries
    rng = np.random.default_rng(7)
    parts = [rng.integers(0, 4, 16000, dtype=np.uint8), np.zeros(3000, dtype=np.uint8),
             np.array([255], dtype=np.uint8), np.tile(np.array([0, 1], dtype=np.uint8), 2500),
             np.array([254], dtype=np.uint8), rng.integers(0, 4, 50000, dtype=np.uint8)]
    t = np.concatenate(parts)
    e = O.Esa(t)
    for minlen in (1, 5, 255, 1000):
        want = _cpu(e, minlen)
        for shards in (1, 3, 7):
            assert np.array_equal(_gpu(e, minlen, shards), want), (minlen, shards)


def test_errors_are_reported():
    e = oracle_esa("Atinsert.fna")
    with pytest.raises(G.SmaxError):
        G.enumerate_smax(e.lcpbytes, e.llv, e.bwt, e.n, e.n + 5, 8)
    with pytest.raises(G.SmaxError):
        G.enumerate_smax(e.lcpbytes, e.llv, e.bwt, e.n, e.nonspecials, 0)


@pytest.mark.parametrize("shards", [1, 3])
def test_inconsistent_llv_is_refused(shards):
    # the .llv scan runs beside the staged upload; no plan is created over
    # tables it rejects, and the call reports the first bad entry (an entry
    # whose position holds no 255 byte, then positions out of order)
    e = oracle_esa("at1MB")
    assert len(e.llv) > 2
    good = e.llv.copy()
    bad = good.copy()
    k = len(bad) // 2
    p = int(bad[k, 0])
    assert e.lcpbytes[p] == 255
    q = next(x for x in range(p + 1, int(bad[k + 1, 0])) if e.lcpbytes[x] != 255) \
        if int(bad[k + 1, 0]) > p + 1 else None
    if q is None:   # no gap to the next entry: move onto a non-255 byte before it
        q = next(x for x in range(p - 1, int(bad[k - 1, 0]), -1) if e.lcpbytes[x] != 255)
    bad[k, 0] = q
    with pytest.raises(G.SmaxError, match="inconsistent .llv entry"):
        G.enumerate_smax(e.lcpbytes, bad, e.bwt, e.n, e.nonspecials, 20, shards)
    bad = good.copy()
    bad[1, 0], bad[2, 0] = good[2, 0], good[1, 0]
    with pytest.raises(G.SmaxError, match="inconsistent .llv entry"):
        G.enumerate_smax(e.lcpbytes, bad, e.bwt, e.n, e.nonspecials, 20, shards)
    # the same call on the good tables still works (state left clean)
    assert np.array_equal(G.enumerate_smax(e.lcpbytes, good, e.bwt, e.n, e.nonspecials, 20, shards),
                          O.linsmax(e.lcpbytes, good, e.bwt, e.nonspecials, 20))


def _triplicated_text(rng, nwords):
    # words occurring three times, each copy closed by a separator: every
    # suffix inside a word shares exactly the rest of the word with its two
    # copies, so a third of the suffix rows are plateaus of 2 rows -- far more
    # exact-evaluation starts per tile than the direct path queues
    parts = []
    for _ in range(nwords):
        w = rng.integers(0, 4, int(rng.integers(24, 40)), dtype=np.uint8)
        for _ in range(3 if rng.random() < 0.8 else 2):
            parts.append(w)
            parts.append(np.array([255], dtype=np.uint8))
    return np.concatenate(parts)


def test_exact_queue_overflow_falls_back():
    rng = np.random.default_rng(11)
    e = O.Esa(_triplicated_text(rng, 1500))
    for minlen in (2, 10, 20):
        want = _cpu(e, minlen)
        for shards in (1, 3):
            assert np.array_equal(_gpu(e, minlen, shards), want), (minlen, shards)


@pytest.mark.parametrize("hook", ["GT_SMAX_ALL_STATIC", "GT_SMAX_BYTE_WINDOWS"])
def test_detection_paths_agree(monkeypatch, hook):
    # plan-time test hooks of the production library: GT_SMAX_ALL_STATIC
    # sends every tile through K1b's exact path, GT_SMAX_BYTE_WINDOWS keeps
    # byte BWT windows instead of packed ones.  Same answers required.
    monkeypatch.setenv(hook, "1")
    e = oracle_esa("at1MB")
    for minlen in (5, 20, 256):
        assert np.array_equal(_gpu(e, minlen, 2), _cpu(e, minlen)), minlen
    rng = np.random.default_rng(5)
    e2 = O.Esa(_repetitive_text(rng, 60000, 0.001))
    for minlen in (3, 20, 300):
        assert np.array_equal(_gpu(e2, minlen), _cpu(e2, minlen)), minlen


def test_runtime_deferrals_past_the_wide_slots():
    """K1's runtime deferral list beyond the plan's wide slots (max(256,
    tiles/256) of them): those K1b tiles take their record runs from the pool
    cursor.  A uniform random text at minlen 2 has hundreds of short
    supermaximal repeats per 2048-row tile, more than a K1 slot holds, so
    every one of its ~730 tiles is deferred at run time; records equal the
    oracle's through the plan and through the host entry point."""
    rng = np.random.default_rng(12)
    t = rng.integers(0, 4, 1_500_000, dtype=np.uint8)
    esa = G.DeviceEsa(t, device=0)
    host = esa.download()
    N = esa.nonspecials
    for minlen in (2, 20):
        want = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], N, minlen)
        p = esa.plan(minlen, capacity=len(want) + 4096)
        p.run()
        got = p.fetch_triples()
        deferred = p.deferred_tiles()
        p.close()
        assert np.array_equal(got, want), minlen
        if minlen == 2:
            assert deferred > 256, deferred
        got = G.enumerate_smax(host["lcptab"], host["llvtab"], host["bwttab"], esa.totallength, N,
                               minlen, 3)
        assert np.array_equal(got, want), minlen
    esa.release()


def test_protein_alphabet_uses_byte_windows():
    # sigma = 20 (not DNA): K1 keeps byte BWT windows
    rng = np.random.default_rng(21)
    fam = [rng.integers(0, 20, int(rng.integers(30, 300)), dtype=np.uint8) for _ in range(8)]
    t = rng.integers(0, 20, 120000, dtype=np.uint8)
    for _ in range(300):
        f = fam[int(rng.integers(0, len(fam)))]
        at = int(rng.integers(0, len(t) - len(f)))
        t[at:at + len(f)] = f
    t[rng.random(len(t)) < 0.002] = 255
    e = O.Esa(t)
    for minlen in (2, 8, 30, 256):
        want = _cpu(e, minlen)
        for shards in (1, 4):
            assert np.array_equal(_gpu(e, minlen, shards), want), (minlen, shards)


def test_result_view_outlives_parent():
    """enumerate_smax hands the C layer's buffer to numpy without a copy:
    views keep it alive, and it is writable and C-contiguous."""
    import gc
    e = oracle_esa("at1MB")
    a = _gpu(e, 20)
    ref = _cpu(e, 20)
    tail = a[-5:]
    col = a[:, 1]
    del a
    gc.collect()
    assert np.array_equal(tail, ref[-5:])
    assert np.array_equal(col, ref[:, 1])
    b = _gpu(e, 20)
    assert b.flags.c_contiguous and b.flags.writeable
    b[0, 0] += 1
    assert b[0, 0] == ref[0, 0] + 1


def test_host_path_multi_chunk_output():
    """> 4 Mi intervals: the pinned D2H runs in several 4 Mi-record chunks
    (and the H2D in many 64 MiB chunks); content equals the CPU oracle."""
    text = G.synth_genome("human", 800_000_000, 3, threads=16)
    esa = G.DeviceEsa(text, device=0, keep_suftab=False)
    host = esa.download()
    n, N = esa.totallength, esa.nonspecials
    esa.release()
    iv = G.enumerate_smax(host["lcptab"], host["llvtab"], host["bwttab"], n, N, 20, 1)
    assert len(iv) > (4 << 20)
    ref = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], N, 20, threads=8)
    assert np.array_equal(iv, ref)


@pytest.mark.parametrize("dense", ["0", "1"])
def test_dense_llv_kernel_variant(monkeypatch, dense):
    # K1's dense-.llv variant (vectorised 255-after-255 relations, chosen by
    # .llv density at plan time) and the default one, forced either way on
    # texts with long repeats (runs of 255 bytes, equal and unequal .llv
    # neighbours) and on at1MB at minlens around 255
    monkeypatch.setenv("GT_SMAX_DENSE", dense)
    rng = np.random.default_rng(77)
    for k in range(3):
        a = rng.integers(0, 4, int(rng.integers(600, 3000)), dtype=np.uint8)
        b = a.copy()
        b[len(b) // 2] = (b[len(b) // 2] + 1) % 4
        parts = [rng.integers(0, 4, 20000, dtype=np.uint8)]
        for _ in range(4 + k):
            parts += [a, rng.integers(0, 4, 50, dtype=np.uint8), b,
                      np.array([255], dtype=np.uint8)]
        t = np.concatenate(parts)
        e = O.Esa(t)
        assert len(e.llv) > 100
        for minlen in (20, 255, 400):
            assert np.array_equal(_gpu(e, minlen), _cpu(e, minlen)), (k, minlen)
    e = oracle_esa("at1MB")
    for minlen in (20, 255, 300):
        assert np.array_equal(_gpu(e, minlen), _cpu(e, minlen)), minlen


def test_width_limits_are_refused():
    """The device record carries a 32-bit lcp (GtSmaxRecord.lcp) and K1 indexes
    a shard's .llv with 32 bits; the reference carries GtUword lcp values
    (src/match/lcpoverflow.h:26-30).  Tables past those widths are refused
    with a message, never truncated: an .llv value >= 2^32 through the plan
    and through the host-table entry point, and more than 2^32 .llv entries
    in one shard through the plan (refused before any kernel reads them)."""
    import torch
    e = oracle_esa("at1MB")
    assert len(e.llv) > 2
    big = e.llv.copy()
    big[len(big) // 2, 1] = (1 << 32) + 7
    with pytest.raises(G.SmaxError, match=r"lcp value >= 2\^32 in \.llv"):
        G.enumerate_smax(e.lcpbytes, big, e.bwt, e.n, e.nonspecials, 20)
    with pytest.raises(G.SmaxError, match=r"lcp value >= 2\^32 in \.llv"):
        G.enumerate_smax(e.lcpbytes, big, e.bwt, e.n, e.nonspecials, 20, 3)

    def padded(a, n):
        t = torch.zeros(G.PAD_FRONT + n + G.PAD_BACK, dtype=torch.uint8, device="cuda")
        t[G.PAD_FRONT:G.PAD_FRONT + len(a)] = torch.from_numpy(np.ascontiguousarray(a))
        return t, t.data_ptr() + G.PAD_FRONT

    N = e.nonspecials
    length = N + 1
    lcp_t, lcp_p = padded(e.lcpbytes[:length], length)
    bwt_t, bwt_p = padded(e.bwt[:length], length)
    llv_t = torch.from_numpy(np.ascontiguousarray(
        np.vstack([big, np.zeros((1, 2), np.uint64)]).view(np.int64))).cuda()
    with pytest.raises(G.SmaxError, match=r"lcp value >= 2\^32 in \.llv"):
        G.SmaxPlan(lcp_p, bwt_p, llv_t.data_ptr(), len(big), 0, length, 1, N, N, 20)
    with pytest.raises(G.SmaxError, match=r"more than 2\^32 \.llv entries"):
        G.SmaxPlan(lcp_p, bwt_p, llv_t.data_ptr(), (1 << 32) + 1, 0, length, 1, N, N, 20)
    # the good tables still plan and run after the refusals
    good_t = torch.from_numpy(np.ascontiguousarray(
        np.vstack([e.llv, np.zeros((1, 2), np.uint64)]).view(np.int64))).cuda()
    p = G.SmaxPlan(lcp_p, bwt_p, good_t.data_ptr(), len(e.llv), 0, length, 1, N, N, 20)
    p.run()
    assert np.array_equal(p.fetch_triples(), _cpu(e, 20))
    p.close()


def test_read_set_keeps_packed_groups_in_k1():
    """Read sets put a separator every few hundred rows, so most K1 windows
    hold a special BWT row; the plan then keeps K1 on the u64 packed groups
    (smax_scan_kernel) instead of sending those windows to K1b with the
    2-plane stream.  Records equal the oracle's either way (GT_SMAX_BW2=1
    forces the 2-plane stream: nearly every tile in K1b)."""
    import os
    rng = np.random.default_rng(31)
    fams = [rng.integers(0, 4, 150, dtype=np.uint8) for _ in range(40)]
    parts = []
    for _ in range(20000):
        r = rng.integers(0, 4, 100, dtype=np.uint8)
        if rng.random() < 0.5:   # reads from shared families: long lcps, smax intervals
            f = fams[int(rng.integers(0, len(fams)))]
            at = int(rng.integers(0, 50))
            r = f[at:at + 100].copy()
            r[rng.random(100) < 0.02] = rng.integers(0, 4, dtype=np.uint8)
        parts += [r, np.array([255], dtype=np.uint8)]
    t = np.concatenate(parts[:-1])
    esa = G.DeviceEsa(t, device=0)
    host = esa.download()
    want = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], esa.nonspecials, 20)
    assert len(want) > 1000
    p = esa.plan(20)
    assert p.scan_kernel() == "smax_scan_kernel", p.scan_kernel()
    p.run()
    assert np.array_equal(p.fetch_triples(), want)
    p.close()
    old = os.environ.get("GT_SMAX_BW2")
    os.environ["GT_SMAX_BW2"] = "1"
    try:
        q = esa.plan(20)
    finally:
        if old is None:
            os.environ.pop("GT_SMAX_BW2", None)
        else:
            os.environ["GT_SMAX_BW2"] = old
    assert q.scan_kernel() == "smax_scan_kernel_b2"
    q.run()
    assert np.array_equal(q.fetch_triples(), want)
    q.close()
    # the host-table entry point chooses the same way (its own staged tables)
    assert np.array_equal(G.enumerate_smax(host["lcptab"], host["llvtab"], host["bwttab"],
                                           esa.totallength, esa.nonspecials, 20, 2), want)
    esa.release()

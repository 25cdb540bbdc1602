"""GPU: the plan-time .llv window index (smax_llv_hist_kernel + the max-scan
launches, csrc/smax_kernels.hip) word for word against its definition.

Tile t of a plan covers rows [g0, g0 + TILE), g0 = base + (tile_first + t)
* TILE; its K1 window stages the .llv entries with positions in
[max(g0 - LH, 0), g0 + TILE + RH).  The word pair K1 reads is {first entry
of the window, entries | left-halo entries << 12 | DMA lanes << 17 | static
<< 31}, static when the window crosses the shard's rows, holds a value >=
2^16, holds more than SMAX_LLV_CAP entries, or (2-plane stream) reads a
packed BWT group holding a special row.  The expected words come from
numpy.searchsorted over the positions -- the two binary searches per tile
the device index replaced -- so a lower bound off by one entry anywhere
fails here, not only where it changes a record.
"""
import numpy as np
import pytest
import torch

import genometools_smax_amd as G
from conftest import oracle_esa
from test_llv_wide_gpu import _dev_padded, _llv_of, _planted

pytestmark = pytest.mark.gpu

TILE, LH, RH, CAP = 2048, 16, 16, 240
STATIC = 1 << 31


def _expected(llv, bwt, length, base, begin, end, bw2):
    tile_first = (begin - base) // TILE
    nt = (end - 1 - base) // TILE - tile_first + 1
    pos = llv[:, 0].astype(np.int64)
    val = llv[:, 1]
    g0 = base + (tile_first + np.arange(nt, dtype=np.int64)) * TILE
    key = np.where(g0 >= LH, g0 - LH, 0)
    lo = np.searchsorted(pos, key, "left")
    lo2 = np.searchsorted(pos, g0 + TILE + RH, "left")
    lo3 = np.searchsorted(pos, g0, "left")
    wide_pre = np.concatenate([[0], np.cumsum(val > 0xFFFF)])
    wide = wide_pre[lo2] - wide_pre[lo] > 0
    wn = lo2 - lo
    halo = lo3 - lo
    stat = (g0 < LH) | (g0 < begin) | (g0 + TILE + RH > end) | wide | (wn + (lo & 7) > CAP)
    if bw2:
        # packed group gi holds local rows 16 (gi - 1) .. 16 (gi - 1) + 15;
        # tile i's window reads groups L/16 .. L/16 + 129, L = (tile_first + i) TILE
        ngroups = length // 16 + 134
        g_lo = tile_first * (TILE // 16)
        g_hi = min(g_lo + nt * (TILE // 16) + 2, ngroups)
        sp_rows = np.flatnonzero(bwt[:length] >= 254)
        for g in np.unique(sp_rows // 16 + 1):
            if not g_lo <= g < g_hi:
                continue
            t_lo = (g - 129 + TILE // 16 - 1) // (TILE // 16) if g >= 129 else 0
            t_hi = g // (TILE // 16)
            for t in range(t_lo, t_hi + 1):
                if tile_first <= t < tile_first + nt:
                    stat[t - tile_first] = True
    nl = np.minimum(np.where(wn == 0, 0, (wn + (lo & 7) + 7) // 8), CAP // 8)
    y = wn | (halo << 12) | (nl << 17) | np.where(stat, STATIC, 0)
    return np.stack([lo.astype(np.uint64), y.astype(np.uint64)], axis=1).astype(np.uint32)


def _check(lcp, llv, bwt, N, ranges, minlen=20):
    length = max(N + 1, len(lcp))
    lcp_t, lcp_p = _dev_padded(lcp, length)
    bwt_t, bwt_p = _dev_padded(bwt, length)
    llv2 = np.zeros((0, 2), np.uint64) if len(llv) == 0 else llv
    llv_t = torch.from_numpy(np.ascontiguousarray(
        np.vstack([llv2, np.zeros((1, 2), np.uint64)]).view(np.int64))).cuda()
    for b, e in ranges:
        p = G.SmaxPlan(lcp_p, bwt_p, llv_t.data_ptr(), len(llv2), 0, length, b, e, N, minlen,
                       capacity=(e - b) // 2 + 4096)
        try:
            got = p.debug_windows()
            bw2 = "_b2" in p.scan_kernel()
            want = _expected(llv2, bwt, length, 0, b, e, bw2)
            assert got.shape == want.shape, (b, e, got.shape, want.shape)
            bad = np.flatnonzero((got != want).any(axis=1))
            assert bad.size == 0, ("range", b, e, "tile", int(bad[0]), got[bad[0]].tolist(),
                                   want[bad[0]].tolist(), bad.size)
        finally:
            p.close()
    del lcp_t, bwt_t, llv_t


def test_index_at1mb_whole_and_ranges():
    e = oracle_esa("at1MB")
    N = e.nonspecials
    ranges = [(1, N), (1, 300001), (300001, 700003), (700003, N), (2047, 2049), (4096, 4097)]
    _check(e.lcpbytes, e.llv, e.bwt, N, ranges)


@pytest.mark.parametrize("seed", [0, 1])
def test_index_planted_wide_values(seed):
    v, bwt, N, edges = _planted(seed)
    lcp, llv = _llv_of(v)
    e1, e2 = edges[len(edges) // 3], edges[2 * len(edges) // 3]
    _check(lcp, llv, bwt, N, [(1, N), (1, e1), (e1, e2), (e2, N)])


def _values(rng, N, at, vals):
    v = rng.integers(0, 200, N + 1).astype(np.uint64)
    v[0] = v[N] = 0
    v[at] = vals
    return v


def test_index_sparse_entries_span_many_tiles():
    # three entries over ~60 tiles: each run of tiles sharing a lower bound
    # is long (one run start per entry, the rest filled by the max-scan)
    rng = np.random.default_rng(5)
    N = 60 * TILE + 77
    v = _values(rng, N, np.array([3, 25 * TILE + 5, 25 * TILE + 2040]), [300, 70000, 255])
    lcp, llv = _llv_of(v)
    bwt = rng.integers(0, 4, N + 1).astype(np.uint8)
    _check(lcp, llv, bwt, N, [(1, N), (TILE + 3, 40 * TILE + 9)])


def test_index_no_entries():
    rng = np.random.default_rng(6)
    N = 20 * TILE + 1
    v = _values(rng, N, np.array([], dtype=np.int64), [])
    lcp, llv = _llv_of(v)
    assert len(llv) == 0
    bwt = rng.integers(0, 4, N + 1).astype(np.uint8)
    _check(lcp, llv, bwt, N, [(1, N), (5 * TILE, 9 * TILE + 1)])


def test_index_dense_window_and_specials():
    # a window with more entries than K1 stages (static by CAP), entries on
    # the halo rows around tile starts, and a few special BWT rows (the
    # 2-plane stream flags the windows reading their groups)
    rng = np.random.default_rng(7)
    N = 30 * TILE + 500
    at = np.concatenate([np.arange(4 * TILE, 4 * TILE + 600),
                         np.array([t * TILE + d for t in range(8, 28, 3) for d in (-17, -16, -1, 0, TILE + 15, TILE + 16)])])
    v = _values(rng, N, np.unique(at), 400)
    lcp, llv = _llv_of(v)
    bwt = rng.integers(0, 4, N + 1).astype(np.uint8)
    bwt[[5, 129 * 16 + 3, 11 * TILE + 7, 20 * TILE - 1]] = 254
    _check(lcp, llv, bwt, N, [(1, N), (3 * TILE + 100, 17 * TILE + 3)])

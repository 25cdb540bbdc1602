"""F2 (maximal pairs) and F3 (lcp-interval tree) past 2^32 suffix rows.

The reference traversal is GtUword throughout (src/match/esa-bottomup.c:
116-273, src/match/esa-maxpairs.c:181-360), so both device paths must cover
every row of a table with more than 2^32 of them: one kernel launch holds
fewer than 2^32 work-items, so their per-row kernels are grid-stride loops
over capped grids (maxpairs.hip MP_FOR, lcpitv.hip LI_FOR).

Tables: N = 2^32 + 2^27 rows, LCP 0 except sparse bumps of 1-3 rows (nested
and flat plateaus, 255 bytes with .llv values, some past row 2^32), random
BWT symbols with specials -- sparse, so that the whole interval list and
pair set fit a host check (the tables need not come from a text: both
algorithms read only the LCP array, the BWT and the suffix array).
  - F3: the device plan's interval list (lcp, lb, rb, father lcp, father
    lb) in pop order equals orc_lcp_intervals (the reference's stack walk)
    exactly;
  - F2: the device plan's pairs (reference emission order) as a set equal
    orc_maxpairs_blocks (the definition, block by block); the suffix array
    is suftab[r] = N - r, so positions map back to rows.
"""
import os

import numpy as np
import pytest
import torch

import genometools_smax_amd as G
import oracle_lib as O

pytestmark = pytest.mark.gpu

N = (1 << 32) + (1 << 27)
CHUNK = 1 << 27


def _sparse_tables(seed=11):
    rng = np.random.default_rng(seed)
    lcp = np.zeros(N + 1, dtype=np.uint8)
    bwt = np.empty(N + 1, dtype=np.uint8)
    llv = []
    for c0 in range(0, N + 1, CHUNK):
        c1 = min(N + 1, c0 + CHUNK)
        m = c1 - c0
        b = bwt[c0:c1]
        b[:] = np.frombuffer(rng.bytes(m), dtype=np.uint8) & 3
        sp = rng.integers(0, m, m // 500)
        b[sp] = 254 + (sp & 1).astype(np.uint8)
        p = np.unique(rng.integers(2, max(3, m - 4), m // 500)) + c0
        p = p[p < N - 3]
        v = rng.integers(1, 61, len(p)).astype(np.uint8)
        lcp[p] = v
        two = p[rng.random(len(p)) < 0.4]
        lcp[two + 1] = np.minimum(lcp[two].astype(np.int64) + rng.integers(0, 31, len(two)), 254)
        three = two[rng.random(len(two)) < 0.35]
        lcp[three + 2] = np.maximum(1, lcp[three] // 2)
        esc = p[rng.random(len(p)) < 0.01]
        lcp[esc] = 255
        llv.append(esc.astype(np.uint64))
    lcp[0] = 0
    lcp[N] = 0
    pos = np.unique(np.concatenate(llv))
    pos = pos[lcp[pos] == 255]
    vals = rng.integers(255, 2000, len(pos)).astype(np.uint64)
    llvtab = np.stack([pos, vals], axis=1).astype(np.uint64)
    assert np.count_nonzero(pos >= 2 ** 32) > 0
    return lcp, llvtab, bwt


@pytest.fixture(scope="module")
def tables():
    return _sparse_tables()


def _dev(lcp, llvtab):
    lcp_t = torch.from_numpy(lcp).to("cuda")
    llv_t = torch.from_numpy(np.ascontiguousarray(
        np.vstack([llvtab, np.zeros((1, 2), np.uint64)])).view(np.int64)).to("cuda")
    return lcp_t, llv_t


def _u64_view(ptr, count):
    """count uint64 of device memory at ptr as a torch view (no copy)."""
    class _View:
        __cuda_array_interface__ = {"shape": (count,), "typestr": "<i8", "data": (ptr, False),
                                    "version": 2}
    return torch.as_tensor(_View(), device="cuda")


def test_lcpitv_intervals_past_2_32(tables):
    lcp, llvtab, _ = tables
    want = O.lcp_intervals(lcp, llvtab, N, cap=N // 100)
    assert np.count_nonzero(want[:, 2] >= 2 ** 32) > 1000
    assert np.count_nonzero(want[:, 0] > 255) > 10
    lcp_t, llv_t = _dev(lcp, llvtab)
    plan = G.LcpitvPlan(lcp_t.data_ptr(), llv_t.data_ptr(), len(llvtab), None, 8, N, device=0)
    n, ptr = plan.intervals()
    assert n == len(want), (n, len(want))
    got = _u64_view(ptr, 5 * n).cpu().numpy().view(np.uint64).reshape(-1, 5)
    plan.close()
    del lcp_t, llv_t
    if not np.array_equal(got, want):
        k = int(np.flatnonzero((got != want).any(axis=1))[0])
        raise AssertionError("first differing record %d: got %s want %s (rows %s)"
                             % (k, got[k].tolist(), want[k].tolist(),
                                lcp[int(want[k][1]):int(want[k][2]) + 2].tolist()))


def test_maxpairs_past_2_32(tables):
    lcp, llvtab, bwt = tables
    minlen = 20
    want = O.maxpairs_blocks(lcp, llvtab, bwt, None, N, minlen, cap=N // 200)
    assert np.count_nonzero(want[:, 2] >= 2 ** 32) > 1000
    lcp_t, llv_t = _dev(lcp, llvtab)
    bwt_t = torch.from_numpy(bwt).to("cuda")
    # suftab[r] = N - r, filled in chunks of 2^30 (one torch.arange over all
    # N + 1 > 2^32 elements left the rows past 2^32 zero on the box)
    suf_t = torch.empty(N + 1, dtype=torch.int64, device="cuda")
    for c0 in range(0, N + 1, 1 << 30):
        c1 = min(N + 1, c0 + (1 << 30))
        suf_t[c0:c1] = torch.arange(N - c0, N - c1, -1, dtype=torch.int64, device="cuda")
    probe = [0, 2 ** 32 - 1, 2 ** 32, 2 ** 32 + 12345, N]
    assert [int(suf_t[r]) for r in probe] == [N - r for r in probe]
    plan = G.MaxpairsPlan(lcp_t.data_ptr(), bwt_t.data_ptr(), llv_t.data_ptr(), len(llvtab),
                          suf_t.data_ptr(), 8, N, minlen, device=0)
    plan.count()
    T = plan.total()
    assert T == len(want), (T, len(want))
    out = torch.empty(3 * T, dtype=torch.int64, device="cuda")
    plan.emit_ordered(out.data_ptr(), T)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint64).reshape(-1, 3).copy()
    # the other ordering path (rank counting with the 4-key split, or the
    # radix passes) on the same pass: the same calls in the same order
    other = "0" if T <= 16384 else str(T)
    old = os.environ.get("GT_MP_RANK_MAX")
    os.environ["GT_MP_RANK_MAX"] = other
    try:
        plan.emit_ordered(out.data_ptr(), T)
        torch.cuda.synchronize()
    finally:
        if old is None:
            os.environ.pop("GT_MP_RANK_MAX")
        else:
            os.environ["GT_MP_RANK_MAX"] = old
    assert np.array_equal(out.cpu().numpy().view(np.uint64).reshape(-1, 3), got)
    plan.close()
    del lcp_t, llv_t, bwt_t, suf_t, out       # the plan borrowed them until here
    # positions -> rows (suftab[r] = N - r); each pair comes in the reference's
    # argument order, compared here as (len, smaller row, larger row)
    r1, r2 = np.uint64(N) - got[:, 1], np.uint64(N) - got[:, 2]
    rows = np.column_stack([got[:, 0], np.minimum(r1, r2), np.maximum(r1, r2)])

    def key(a):
        return a[np.lexsort(a.T[::-1])]
    assert np.array_equal(key(rows), key(want))

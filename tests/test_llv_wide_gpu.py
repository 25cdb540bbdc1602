"""GPU parity on the `.llv` u16-overflow route: LCP values >= 65,536.

K1 stages a window's `.llv` values as u16 (smax_kernels.hip: issue_lcp_llv,
smax_llv16_kernel); a window holding a value above 0xffff is flagged static
at plan time (smax_llv_index_kernel) and decided exactly by K1b from the
full `.llv` records.  The reference carries GtUword values through the same
255 -> `.llv` decode (/root/reference/src/match/lcpoverflow.h:23-30,
/root/reference/src/match/esa-seqread.h:160), so every value here must come
out exactly as the oracle's linear scan (orc_linsmax) sees it.

Two kinds of input:
  - planted tables: random small LCP bytes with `.llv` values 65,535,
    65,536, 65,537, 131,072 ... placed on tile and window edges (rows
    k*2048 - 16 .. k*2048 + 16) in the relations a u16 truncation would
    flip (65,535 -> 65,536 reads as a descent, 300 -> 65,836 as a plateau,
    131,072 -> 65,536 as equal), plateaus of big values across a tile edge
    and across shard edges;
  - a real ESA (the GPU suffixerator, byte-identical to the oracle's
    restatement) of a text with a 70 kb exact duplicate, duplicates of
    exactly 65,535 and 65,536 bases, and a 70 kb homopolymer.
Each runs through gt_smax_plan_create (one plan, and three range plans with
the device stitch) and through gt_smax_hip_enumerate_to_buffer (1 and 3
shards), at minlen 20, 255 and 65,535.
"""
import numpy as np
import pytest
import torch

import genometools_smax_amd as G
import oracle_lib as O

pytestmark = pytest.mark.gpu

TILE = 2048
MINLENS = (20, 255, 65535)


def _llv_of(values):
    """(lcp bytes, .llv records) of exact LCP values (GtSmaxLlv layout)."""
    values = np.asarray(values, dtype=np.uint64)
    lcp = np.minimum(values, 255).astype(np.uint8)
    pos = np.flatnonzero(values >= 255).astype(np.uint64)
    llv = np.stack([pos, values[pos]], axis=1) if len(pos) else np.zeros((0, 2), np.uint64)
    return lcp, np.ascontiguousarray(llv, dtype=np.uint64)


def _planted(seed, ntiles=24):
    """Tables of N = ntiles * 2048 + 777 rows with big `.llv` values on edges.

    Returns (exact LCP values, BWT bytes, N, shard ends inside big plateaus)."""
    rng = np.random.default_rng(seed)
    N = ntiles * TILE + 777
    v = rng.integers(0, 40, N + 1).astype(np.uint64)
    v[0] = 0
    v[N] = 0
    bwt = rng.integers(0, 4, N + 1).astype(np.uint8)
    bwt[N] = 254

    def put(row, vals, distinct=True):
        vals = np.asarray(vals, dtype=np.uint64)
        v[row:row + len(vals)] = vals
        if distinct:
            # the interval's rows [row-1, row+len) get pairwise distinct left
            # symbols (ACGT, then specials, which are unique): accepted records
            k = len(vals) + 1
            sym = np.array([0, 1, 2, 3] + [254] * max(0, k - 4), dtype=np.uint8)[:k]
            bwt[row - 1:row - 1 + k] = rng.permutation(sym)

    edges = []
    patterns = [
        [65535, 65536],                  # u16: 65535 -> 0, a false descent
        [65536, 65535],
        [300, 65836, 300],               # u16: 300 == 300, a false plateau
        [131072, 65536, 30],             # u16: 0 == 0
        [65536, 65536, 65536],           # a 3-row plateau of one big value
        [65537],
        [70000, 70000, 70000, 70000, 70000, 70000],   # plateau across the edge
        [65535],
        [255, 65535, 65535, 256],
    ]
    offsets = [-16, -9, -3, -2, -1, 0, 1, 5, 2040, 16]
    for t in range(1, ntiles):
        g0 = t * TILE
        pat = patterns[t % len(patterns)]
        off = offsets[t % len(offsets)]
        row = g0 + off - (len(pat) // 2 if off in (-1, 0, 1) else 0)
        # a smaller LCP on both sides: local maxima (records) where diverse
        v[row - 1] = 10
        v[row + len(pat)] = 12
        put(row, pat, distinct=(t % 3 != 0))
        edges.append(row + len(pat) // 2)
    # values of exactly 65,535 / 65,536 on the halo rows of one window
    for t, val in ((5, 65535), (6, 65536), (7, 65536), (8, 65535)):
        g0 = t * TILE
        for r in (g0 - 16, g0 + TILE + 15):
            v[r] = val
    return v, bwt, N, edges


def _dev_padded(a, length):
    t = torch.zeros(G.PAD_FRONT + length + G.PAD_BACK, dtype=torch.uint8, device="cuda")
    t[G.PAD_FRONT:G.PAD_FRONT + len(a)] = torch.from_numpy(np.ascontiguousarray(a))
    return t, t.data_ptr() + G.PAD_FRONT


def _plan_runs(lcp, llv, bwt, N, minlen, ranges):
    """Range plans over the whole device tables: part 0, boundary into the
    gathered buffer, part 1, device stitch; records concatenated."""
    length = max(N + 1, len(lcp))   # multi-sequence tables: n + 1 > N + 1
    lcp_t, lcp_p = _dev_padded(lcp, length)
    bwt_t, bwt_p = _dev_padded(bwt, length)
    llv_t = torch.from_numpy(np.ascontiguousarray(
        np.vstack([llv, np.zeros((1, 2), np.uint64)]).view(np.int64))).cuda()
    world = len(ranges)
    gathered = torch.zeros(G.BOUNDARY_BYTES * world, dtype=torch.uint8, device="cuda")
    plans = []
    for r, (b, e) in enumerate(ranges):
        # random small LCP bytes make far more records than the default
        # capacity ((end - begin) / 64) assumes: one per two rows at most
        p = G.SmaxPlan(lcp_p, bwt_p, llv_t.data_ptr(), len(llv), 0, length, b, e, N, minlen,
                       capacity=(e - b) // 2 + 4096)
        p.run_part(0)
        p.copy_boundary(gathered.data_ptr() + G.BOUNDARY_BYTES * r)
        p.run_part(1)
        plans.append(p)
    torch.cuda.synchronize()
    parts = []
    for r, p in enumerate(plans):
        if world > 1:
            p.stitch(gathered.data_ptr(), world, r)
        parts.append(p.fetch_triples())
        assert p.error_bits() == 0
        p.close()
    del lcp_t, bwt_t, llv_t
    return np.concatenate(parts) if parts else np.zeros((0, 3), np.uint64)


def _check_all(lcp, llv, bwt, n, N, shard_ends, label):
    for minlen in MINLENS:
        want = O.linsmax(lcp, llv, bwt, N, minlen)
        if minlen <= 65535:
            assert np.count_nonzero(want[:, 0] >= 65535) > 0, (label, minlen)
        got = _plan_runs(lcp, llv, bwt, N, minlen, [(1, N)])
        assert np.array_equal(got, want), (label, "plan", minlen, len(got), len(want))
        e1, e2 = shard_ends
        got = _plan_runs(lcp, llv, bwt, N, minlen, [(1, e1), (e1, e2), (e2, N)])
        assert np.array_equal(got, want), (label, "3 plans", minlen, len(got), len(want))
        for shards in (1, 3):
            got = G.enumerate_smax(lcp, llv, bwt, n, N, minlen, shards)
            assert np.array_equal(got, want), (label, "host", shards, minlen, len(got), len(want))


@pytest.mark.parametrize("seed", [0, 1])
def test_planted_wide_values_on_tile_edges(seed):
    v, bwt, N, edges = _planted(seed)
    lcp, llv = _llv_of(v)
    assert int(v.max()) >= 131072 and np.count_nonzero(v == 65536) > 3 and np.count_nonzero(v == 65535) > 3
    # the two inner shard ends land inside planted big-value runs
    e1, e2 = edges[len(edges) // 3], edges[2 * len(edges) // 3]
    _check_all(lcp, llv, bwt, N, N, (e1, e2), "planted%d" % seed)


def test_planted_dense_run_of_wide_values():
    # a whole window of 255 bytes whose values climb through 65,536 (a ramp:
    # every row a start, one local maximum) next to one that is flat at 65,536
    rng = np.random.default_rng(9)
    N = 12 * TILE
    v = rng.integers(0, 30, N + 1).astype(np.uint64)
    v[0] = v[N] = 0
    bwt = rng.integers(0, 4, N + 1).astype(np.uint8)
    a = 3 * TILE - 700
    v[a:a + 1400] = np.arange(65536 - 700, 65536 + 700, dtype=np.uint64)
    b = 6 * TILE - 5
    v[b:b + TILE + 10] = 65536
    bwt[b - 1:b + TILE + 10] = 254
    lcp, llv = _llv_of(v)
    _check_all(lcp, llv, bwt, N, N, (a + 699, b + 1000), "ramp")


def _real_text():
    rng = np.random.default_rng(2024)

    def rnd(k):
        return rng.integers(0, 4, k, dtype=np.uint8)

    x70 = rnd(70000)
    x65535 = rnd(65535)
    x65536 = rnd(65536)
    parts = []
    # each copy pair: different left symbols (left-diverse) and different
    # right symbols, so the pair's LCP is exactly the copy's length
    for x in (x70, x65535, x65536):
        for k in range(2):
            parts += [rnd(3000), np.array([k], np.uint8), x, np.array([2 + k], np.uint8)]
    parts += [rnd(2000), np.array([1], np.uint8), np.zeros(70000, np.uint8), np.array([3], np.uint8),
              rnd(5000)]
    return np.concatenate(parts)


def test_real_esa_with_long_duplicates_and_homopolymer():
    text = _real_text()
    esa = G.DeviceEsa(text, device=0)
    host = esa.download()
    n, N = esa.totallength, esa.nonspecials
    lcp, llv, bwt = host["lcptab"], host["llvtab"], host["bwttab"]
    assert int(llv[:, 1].max()) >= 69999
    assert np.count_nonzero(llv[:, 1] == 65535) >= 1 and np.count_nonzero(llv[:, 1] == 65536) >= 1
    want = O.linsmax(lcp, llv, bwt, N, 20)
    exact = set(int(x) for x in want[:, 0])
    assert {65535, 65536, 70000} <= exact, sorted(x for x in exact if x > 60000)
    # the device plan over the builder's own tables (packed BWT)
    for minlen in MINLENS:
        p = esa.plan(minlen)
        p.run()
        got = p.fetch_triples()
        p.close()
        assert np.array_equal(got, O.linsmax(lcp, llv, bwt, N, minlen)), minlen
    esa.release()
    # shard ends inside the big duplicates' rows: the rows of the 70 kb pair
    big = np.flatnonzero(lcp == 255)
    e1, e2 = int(big[len(big) // 3]), int(big[2 * len(big) // 3])
    _check_all(lcp, llv, bwt, n, N, (e1, e2), "real")


def test_plateau_wider_than_65535_rows(tmp_path):
    """An interval of 70,000 rows: 70,000 sequences that are the same
    30-mer, each between two separators (unique left and right symbols), so
    [lb, lb+69,999] with lcp-value 30 is one supermaximal repeat whose width
    does not fit K1's 16-bit result field -- K1 flags the tile wide and K1b
    decides it.  Whole plan, three range plans with shard ends inside the
    plateau (device stitch), host entry with 1 and 3 shards."""
    rng = np.random.default_rng(5)
    acgt = np.frombuffer(b"ACGT", np.uint8)
    motif = acgt[rng.integers(0, 4, 30)].tobytes().decode()
    recs = [">r%d\n%s\n" % (i, acgt[rng.integers(0, 4, 3000)].tobytes().decode()) for i in range(3)]
    recs += [">m%d\n%s\n" % (i, motif) for i in range(70000)]
    recs += [">t\n%s\n" % acgt[rng.integers(0, 4, 5000)].tobytes().decode()]
    text, _ = G.encode_fasta("".join(recs).encode())
    esa = G.DeviceEsa(text, device=0)
    host = esa.download()
    n, N = esa.totallength, esa.nonspecials
    esa.release()
    lcp, llv, bwt = host["lcptab"], host["llvtab"], host["bwttab"]
    want20 = O.linsmax(lcp, llv, bwt, N, 20)
    wid = want20[:, 2] - want20[:, 1] + 1
    assert int(wid.max()) == 70000 and int(want20[wid.argmax(), 0]) == 30
    lb = int(want20[wid.argmax(), 1])
    e1, e2 = lb + 20000, lb + 50000
    for minlen in (20, 30, 31):
        want = O.linsmax(lcp, llv, bwt, N, minlen)
        got = _plan_runs(lcp, llv, bwt, N, minlen, [(1, N)])
        assert np.array_equal(got, want), ("plan", minlen, len(got), len(want))
        got = _plan_runs(lcp, llv, bwt, N, minlen, [(1, e1), (e1, e2), (e2, N)])
        assert np.array_equal(got, want), ("3 plans", minlen, len(got), len(want))
        for shards in (1, 3):
            got = G.enumerate_smax(lcp, llv, bwt, n, N, minlen, shards)
            assert np.array_equal(got, want), ("host", shards, minlen, len(got), len(want))

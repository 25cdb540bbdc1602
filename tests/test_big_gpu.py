"""Past 2^32 suffixes on the GPU (BASELINE config C5's 64-bit path):

  - a 4.4 Gbp human-like genome (n + 1 > 2^32 rows, .llv entries past
    2^32) built whole by the 64-bit ESA builder: the smax plan's interval
    array equals the all-core CPU oracle's over every row, and so does the
    host-table entry point with 3 shards;
  - windows of the same suffix array built as row ranges (around row 2^32,
    at the end, in the middle) are checked against the text itself:
    adjacent suffixes strictly ascending in gt's order (specials unique,
    ranked by position, after every base), every LCP value exact, BWT =
    text[SA-1] (254 for suffix 0) -- the suffixerator contract, size
    independent;
  - synthetic .lcp/.llv/.bwt tables of 2^32 + 2^27 rows (tools/
    big_rows_check.py's generator) through the host entry point, 1 and 3
    shards, against the oracle.
"""
import os
import sys

import numpy as np
import pytest

import genometools_smax_amd as G
import oracle_lib as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def human44():
    text = G.synth_genome("human", 4_400_000_000, 4, threads=16)
    assert len(text) + 1 > 2 ** 32
    return text


def test_whole_build_past_2_32(human44):
    text = human44
    esa = G.DeviceEsa64(text, device=0)
    n, N = esa.totallength, esa.nonspecials
    assert n + 1 > 2 ** 32 and N > 2 ** 32
    p = esa.plan(20)
    p.run()
    cnt = p.fetch_count()
    if cnt + 1 > p.capacity:
        p.close()
        p = esa.plan(20, capacity=cnt + 16)
        p.run()
    got = p.fetch_triples()
    p.close()
    host = esa.download()
    esa.release()
    assert np.count_nonzero(host["llvtab"][:, 0] >= 2 ** 32) > 0
    want = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], N, 20, threads=16)
    assert np.count_nonzero(want[:, 2] >= 2 ** 32) > 1000
    assert np.array_equal(got, want), (len(got), len(want))
    del got
    got = G.enumerate_smax(host["lcptab"], host["llvtab"], host["bwttab"], n, N, 20, 3)
    assert np.array_equal(got, want)


def _check_window(text, lo, hi, d):
    """Suffixerator contract on rows [lo, hi) of the built arrays."""
    n = len(text)
    sa = d["suftab"].astype(np.int64)
    lcp = d["lcptab"].astype(np.int64)
    llv = {int(p): int(v) for p, v in d["llvtab"]}
    exact = np.array([llv[lo + i] if lcp[i] == 255 else lcp[i] for i in range(len(lcp))], dtype=np.int64)
    # BWT
    b = np.where(sa == 0, 254, text[np.maximum(sa - 1, 0)])
    assert np.array_equal(b.astype(np.uint8), d["bwttab"])
    # adjacent pairs (rows lo+1 .. hi-1): walk the common prefix
    a, c = sa[:-1].copy(), sa[1:].copy()
    k = np.zeros(len(a), dtype=np.int64)
    idx = np.arange(len(a))
    done = np.zeros(len(a), dtype=bool)
    less = np.zeros(len(a), dtype=bool)
    pad = np.concatenate([text, np.full(1, 255, np.uint8)])   # position n: end of text (special)
    while not done.all():
        i = idx[~done]
        pa, pc = a[i] + k[i], c[i] + k[i]
        ta = np.where(pa >= n, 256, pad[np.minimum(pa, n)].astype(np.int64))
        tc = np.where(pc >= n, 256, pad[np.minimum(pc, n)].astype(np.int64))
        spa, spc = ta >= 254, tc >= 254
        stop = spa | spc | (ta != tc)
        j = i[stop]
        # order at the first difference: bases < specials; two specials by position
        sa_, sc_ = spa[stop], spc[stop]
        less[j] = np.where(sa_ & sc_, pa[stop] < pc[stop],
                           np.where(sa_ | sc_, ~sa_, ta[stop] < tc[stop]))
        done[j] = True
        k[i[~stop]] += 1
    assert less.all()
    assert np.array_equal(k, exact[1:])


@pytest.mark.parametrize("where", ["at_2_32", "end", "middle"])
def test_range_windows_past_2_32_against_text(human44, where):
    text = human44
    m = len(text) + 1
    lo = {"at_2_32": 2 ** 32 - 40_000, "end": m - 60_000, "middle": m // 2}[where]
    hi = min(m, lo + 80_000)
    esa = G.DeviceEsa64(text, device=0, row_lo=lo, row_hi=hi, keep_suftab=True)
    d = esa.download(suftab=True)
    esa.release()
    _check_window(text, lo, hi, d)


def test_synthetic_tables_past_2_32():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import big_rows_check as B
    lcp, llv, bwt = B.make_tables()
    ref = B.oracle(lcp, llv, bwt)
    assert np.count_nonzero(ref[:, 2] >= 2 ** 32) > 0
    for shards in (1, 3):
        got = G.enumerate_smax(lcp, llv, bwt, B.N, B.N, B.MINLEN, shards)
        assert np.array_equal(got, ref), shards

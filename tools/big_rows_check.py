"""64-bit row path check: N = 2^32 + 2^27 suffix positions (C5 evidence).

Synthetic .lcp/.llv/.bwt tables past the 32-bit row boundary: background
lcp 0..11, ~0.15% bumps of 20..59 (1-3-row plateaus), a sprinkling of
255-escaped .llv values (some at positions >= 2^32) and BWT symbols 0..3
with a few specials.  The HIP path (1 and 3 shards) must return exactly the
oracle's orc_linsmax intervals.  Test infrastructure (uses oracle/).

  python tools/big_rows_check.py > big_rows.json
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import genometools_smax_amd as G  # noqa: E402
import oracle_lib as O  # noqa: E402

N = (1 << 32) + (1 << 27)      # totallength == nonspecials; tables hold N+1 entries
MINLEN = 20
CHUNK = 1 << 27


def _some(rng, m, frac):
    """Sorted distinct positions in [0, m), about frac * m of them."""
    return np.unique(rng.integers(0, m, rng.binomial(m, frac)))


def make_tables(seed=7):
    rng = np.random.default_rng(seed)
    lcp = np.zeros(N + 1, dtype=np.uint8)
    bwt = np.zeros(N + 1, dtype=np.uint8)
    llv_pos = []
    for ci, c0 in enumerate(range(0, N, CHUNK)):
        c1 = min(N, c0 + CHUNK)
        m = c1 - c0
        lc = lcp[c0:c1]
        lc[:] = rng.integers(0, 12, m, dtype=np.uint8)
        bumps = _some(rng, m - 2, 0.0015)
        lc[bumps] = rng.integers(MINLEN, 60, len(bumps), dtype=np.uint8)
        wide = bumps[rng.random(len(bumps)) < 0.3]
        lc[wide + 1] = lc[wide]
        wider = wide[rng.random(len(wide)) < 0.3]
        lc[wider + 2] = lc[wider]
        esc = _some(rng, m, 2e-6)
        lc[esc] = 255
        llv_pos.append(esc.astype(np.uint64) + np.uint64(c0))
        b = bwt[c0:c1]
        b[:] = rng.integers(0, 4, m, dtype=np.uint8)
        sp = _some(rng, m, 0.001)
        b[sp] = rng.integers(254, 256, len(sp), dtype=np.uint8)
        if ci % 8 == 7:
            print(json.dumps({"progress": "chunk", "rows": int(c1)}), file=sys.stderr, flush=True)
    pos = np.concatenate(llv_pos)
    if len(pos) and pos[0] == 0:
        pos = pos[1:]
    lcp[0] = 0
    lcp[N] = 0
    llv = np.empty((len(pos), 2), dtype=np.uint64)
    llv[:, 0] = pos
    llv[:, 1] = np.random.default_rng(seed + 1).integers(255, 2000, len(pos), dtype=np.uint64)
    return lcp, llv, bwt


def oracle(lcp, llv, bwt, cap=40_000_000):
    out = np.empty(3 * cap, dtype=np.uint64)
    found = O.lib().orc_linsmax(O._p(lcp, O._u8p), llv.ctypes.data_as(ctypes.c_void_p), len(llv),
                                O._p(bwt, O._u8p), N, MINLEN, O._p(out, O._u64p), cap)
    assert found <= cap, found
    return out[: 3 * found].reshape(-1, 3)


def main():
    t0 = time.time()
    lcp, llv, bwt = make_tables()
    rep = {"n": N, "minlen": MINLEN, "numllv": int(len(llv)),
           "llv_above_2^32": int(np.count_nonzero(llv[:, 0] >= (1 << 32))),
           "gen_s": round(time.time() - t0, 1)}
    print(json.dumps({"progress": "tables", **rep}), file=sys.stderr, flush=True)
    t0 = time.time()
    ref = oracle(lcp, llv, bwt)
    rep["oracle_s"] = round(time.time() - t0, 1)
    rep["intervals"] = int(len(ref))
    rep["intervals_rb_above_2^32"] = int(np.count_nonzero(ref[:, 2] >= (1 << 32)))
    rep["llv_intervals"] = int(np.count_nonzero(ref[:, 0] >= 255))
    print(json.dumps({"progress": "oracle", "intervals": len(ref)}), file=sys.stderr, flush=True)
    for shards in (1, 3):
        t0 = time.time()
        got = G.enumerate_smax(lcp, llv, bwt, N, N, MINLEN, shards)
        rep["hip_s_shards_%d" % shards] = round(time.time() - t0, 1)
        rep["identical_shards_%d" % shards] = bool(got.shape == ref.shape and np.array_equal(got, ref))
        print(json.dumps({"progress": "hip", "shards": shards}), file=sys.stderr, flush=True)
        del got
    print(json.dumps(rep))
    sys.exit(0 if rep["identical_shards_1"] and rep["identical_shards_3"] else 1)


if __name__ == "__main__":
    main()

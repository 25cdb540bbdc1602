"""The emission-order rule the GPU maxpairs pass sorts by (csrc/maxpairs.hip
header), restated in Python and checked against the oracle's restatement of
the reference traversal (orc_maxpairs, which reproduces the reference's
testdata/repfind-8-Atinsert.txt line for line): sorting the oracle's pairs
by the rule's keys must leave them in the order the traversal emitted them.

Rule (rows x < y, pair depth L, t = min{k >= y : LCP[k+1] <= L}):
events by (t, -L); inside an event, for the leaf event
(max(LCP[y], LCP[y+1]) == L) by (class x, x), for a branch event by
(class x, class y, x, y) / (class x, 254, y, x) / (254, x, class y, y),
class = BWT symbol, 254 for every symbol >= 254.
"""
import numpy as np
import pytest

import oracle_lib as O
from conftest import oracle_esa


def _rule_order(e, pairs):
    N = e.nonspecials
    X = e.lcp.astype(np.int64).copy()
    X[0] = 0
    X[N] = 0
    inv = np.empty(e.n + 1, dtype=np.int64)
    inv[e.suftab.astype(np.int64)] = np.arange(e.n + 1)
    keys = []
    for k, (depth, p1, p2) in enumerate(pairs):
        x, y = sorted((int(inv[p1]), int(inv[p2])))
        depth = int(depth)
        t = y
        while X[t + 1] > depth:
            t += 1
        cx = min(int(e.bwt[x]), 254)
        cy = min(int(e.bwt[y]), 254)
        if max(X[y], X[y + 1]) == depth:
            w = (cx, 0, x, 0)
        elif cx < 254 and cy < 254:
            w = (cx, cy, x, y)
        elif cx < 254:
            w = (cx, 254, y, x)
        else:
            w = (254, 0, x, (cy << 40) | y)
        keys.append((t, -depth) + w + (k,))
    keys.sort()
    return [k[-1] for k in keys]


@pytest.mark.parametrize("seed", range(3))
def test_rule_reproduces_traversal_order(seed):
    rng = np.random.default_rng(500 + seed)
    for _ in range(40):
        n = int(rng.integers(2, 300))
        t = rng.integers(0, int(rng.integers(1, 5)), n, dtype=np.uint8)
        if rng.random() < 0.5:
            t[rng.random(n) < 0.1] = rng.choice(np.array([254, 255], np.uint8))
        e = O.Esa(t)
        for minlen in (1, 2, 4):
            p = O.maxpairs(e, minlen)
            assert _rule_order(e, p) == list(range(len(p))), (n, minlen)


@pytest.mark.parametrize("minlen", [4, 8])
def test_rule_on_atinsert(minlen):
    e = oracle_esa("Atinsert.fna")
    p = O.maxpairs(e, minlen)
    assert len(p) > 400
    assert _rule_order(e, p) == list(range(len(p)))

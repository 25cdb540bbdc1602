"""GPU parity at BASELINE.json's own configurations, bit for bit.

C2 (configs[1]): 100 Mbp uniform i.i.d. ACGT, seed 42, minlen 20.
C3 (configs[2]): 3 Gbp synthetic human-like genome, seed 1, minlen 20.

Each genome is built into HBM by the repo's GPU suffixerator replacement
(the setup bench.py uses), and the full (lcp, lb, rb) interval arrays of
  - the device-resident plan (the path bench.py times), and
  - the host-table drop-in boundary (gt_smax_hip_enumerate_to_buffer)
are compared with the CPU oracle's linear A10 scan over the same tables
(orc_linsmax; orc_linsmax_mt with 16 threads at 3 Gbp -- same output,
tests/test_oracle.py pins the two against each other).
"""
import numpy as np
import pytest

import genometools_smax_amd as G
import oracle_lib as O

pytestmark = pytest.mark.gpu


def _config_case(kind, bases, seed, minlen, threads):
    text = G.synth_genome(kind, bases, seed, threads=16)
    esa = G.DeviceEsa(text, device=0, keep_suftab=False)
    del text
    n, N = esa.totallength, esa.nonspecials
    plan = esa.plan(minlen)
    plan.run()
    cnt = plan.fetch_count()
    if cnt > plan.capacity:
        plan.close()
        plan = esa.plan(minlen, capacity=cnt + 16)
        plan.run()
    dev = plan.fetch_triples()
    plan.close()
    host = esa.download()
    esa.release()
    want = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], N, minlen, threads=threads)
    assert len(want) > 0
    assert np.array_equal(dev, want), (len(dev), len(want))
    del dev
    got = G.enumerate_smax(host["lcptab"], host["llvtab"], host["bwttab"], n, N, minlen, 1)
    assert np.array_equal(got, want), (len(got), len(want))
    return N, len(want)


def test_c2_uniform_100mbp():
    N, k = _config_case("uniform", 100_000_000, 42, 20, 1)
    assert N == 100_000_000
    assert k > 1000


def test_c3_human_like_3gbp():
    N, k = _config_case("human", 3_000_000_000, 1, 20, 16)
    assert N > 2_900_000_000
    assert k > 10_000_000

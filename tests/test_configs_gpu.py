"""GPU parity at BASELINE.json's own configurations, bit for bit.

C2 (configs[1]): 100 Mbp uniform i.i.d. ACGT, seed 42, minlen 20.
C3 (configs[2]): 3 Gbp synthetic human-like genome, seed 1, minlen 20.
C4 (configs[3]): C3's suffix array range-sharded 8 ways as bench.py --gpus 8
    runs it (one process per GPU there; here the 8 ranks run in turn on one
    GPU): each rank builds only rows [begin-1, end+1) with the 64-bit range
    builder, enqueues the scan (part 0), puts its 152-byte boundary record
    into the gathered buffer (the RCCL all-gather's output layout), runs the
    compaction (part 1), and stitches from the gathered records; the ranks'
    record lists concatenated in rank order equal the whole-table oracle.
C5 (configs[4]): 12 Gbp synthetic plant-like genome, seed 2, minlen 50 --
    11.9e9 suffixes, the 64-bit suftab path (the reference's suffix width
    rule, src/match/sfx-suffixgetset.c:48-51), built whole on one GPU.

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
import torch

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


def test_c4_eight_way_split_3gbp():
    world, minlen = 8, 20
    text = G.synth_genome("human", 3_000_000_000, 1, threads=16)
    n = len(text)
    N = n - int(np.count_nonzero(text >= 254))
    gathered = torch.zeros(G.BOUNDARY_BYTES * world, dtype=torch.uint8, device="cuda")
    esas, plans = [], []
    for r in range(world):
        begin = 1 + (N - 1) * r // world          # bench.py's split rule
        end = 1 + (N - 1) * (r + 1) // world
        e = G.DeviceEsa64(text, device=0, row_lo=begin - 1, row_hi=end + 1)
        p = e.plan(minlen, begin, end, capacity=(end - begin) // 8 + 4096)
        p.run_part(0)
        p.copy_boundary(gathered.data_ptr() + G.BOUNDARY_BYTES * r)
        p.run_part(1)
        esas.append(e)
        plans.append(p)
    torch.cuda.synchronize()
    parts = []
    for r, p in enumerate(plans):
        p.stitch(gathered.data_ptr(), world, r)
        assert p.fetch_count() <= p.capacity
        parts.append(p.fetch_triples())
        p.close()
    for e in esas:
        e.release()
    got = np.concatenate(parts)
    del parts
    full = G.DeviceEsa(text, device=0, keep_suftab=False)
    del text
    assert full.nonspecials == N
    host = full.download()
    full.release()
    want = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], N, minlen, threads=16)
    assert len(want) > 10_000_000
    assert np.array_equal(got, want), (len(got), len(want))


def test_c5_plant_12gbp():
    minlen = 50
    text = G.synth_genome("plant", 12_000_000_000, 2, threads=16)
    n = len(text)
    esa = G.DeviceEsa64(text, device=0)
    del text
    N = esa.nonspecials
    assert n + 1 > 2 ** 32 and N > 2 ** 33
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
    want = O.linsmax(host["lcptab"], host["llvtab"], host["bwttab"], N, minlen, threads=16)
    assert len(want) > 10_000_000
    assert np.count_nonzero(want[:, 2] >= 2 ** 32) > len(want) // 2
    assert np.array_equal(dev, want), (len(dev), len(want))
    del dev
    # the host-table drop-in boundary over the same 12 Gbp tables, 2 shards
    got = G.enumerate_smax(host["lcptab"], host["llvtab"], host["bwttab"], n, N, minlen, 2)
    assert np.array_equal(got, want), (len(got), len(want))

"""GPU parity of the 64-bit, range-restricted ESA builder (esa_build64.hip,
gt_smax_esa64_build) -- the producer of BASELINE config C5 (12 Gbp, > 2^32
suffixes) and of the per-rank suffix-array ranges of a multi-GPU run.

  - byte-identical tables (.lcp, .llv, .bwt, the packed BWT, the 8-byte
    suffix array) to the oracle's suffixerator restatement on the reference
    fixtures and to the 32-bit GPU builder on synthetic genomes, with one
    batch and with many (batch_max);
  - a range build equals the same rows of the full build;
  - smax over three range-built shards (plans + device boundary stitch)
    equals the CPU oracle's answer over the full tables.
"""
import numpy as np
import pytest
import torch

import genometools_smax_amd as G
import oracle_lib as O
from conftest import oracle_esa

pytestmark = pytest.mark.gpu


def _full(text, **kw):
    e = G.DeviceEsa64(text, device=0, keep_suftab=True, **kw)
    d = e.download(suftab=True)
    info = (e.totallength, e.nonspecials, e.numllv, e.esa.batches)
    e.release()
    return d, info


@pytest.mark.parametrize("name,batch_max", [("Atinsert.fna", 0), ("Atinsert.fna", 6000),
                                            ("at1MB", 0), ("at1MB", 120_000)])
def test_fixture_tables_equal_oracle(name, batch_max):
    e = oracle_esa(name)
    d, (n, N, nllv, batches) = _full(e.text, batch_max=batch_max)
    assert n == e.n and N == e.nonspecials
    if batch_max:
        assert batches > 1
    assert np.array_equal(d["lcptab"], e.lcpbytes)
    assert np.array_equal(d["bwttab"], e.bwt)
    assert np.array_equal(d["llvtab"], e.llv.reshape(-1, 2))
    assert np.array_equal(d["suftab"], e.suftab.astype(np.uint64))
    assert np.array_equal(d["bwtpk"], O.pack_bwt_ref(e.bwt)[0])


@pytest.mark.parametrize("kind,bases,seed,batch_max", [("human", 20_000_000, 3, 0),
                                                       ("human", 20_000_000, 3, 4_000_000),
                                                       ("plant", 12_000_000, 2, 3_000_000),
                                                       ("uniform", 5_000_000, 9, 1_000_000)])
def test_equals_32bit_builder(kind, bases, seed, batch_max):
    text = G.synth_genome(kind, bases, seed, threads=8)
    e32 = G.DeviceEsa(text, device=0, keep_suftab=True)
    want = e32.download(suftab=True)
    want_pk = e32.packed_bwt()
    e32.release()
    got, (n, N, _, batches) = _full(text, batch_max=batch_max)
    assert N == e32.nonspecials
    for k in ("lcptab", "bwttab", "llvtab", "suftab"):
        assert np.array_equal(got[k], want[k]), k
    assert np.array_equal(got["bwtpk"], want_pk)


def test_range_build_equals_full_rows():
    text = G.synth_genome("human", 8_000_000, 11, threads=8)
    full, (n, N, _, _) = _full(text)
    m = n + 1
    for lo, hi in [(0, m // 3), (m // 3, 2 * m // 3 + 5), (2 * m // 3, m), (12345, 12346 + 70_000)]:
        e = G.DeviceEsa64(text, device=0, row_lo=lo, row_hi=hi, keep_suftab=True, batch_max=1_500_000)
        d = e.download(suftab=True)
        e.release()
        assert np.array_equal(d["lcptab"], full["lcptab"][lo:hi])
        assert np.array_equal(d["bwttab"], full["bwttab"][lo:hi])
        assert np.array_equal(d["suftab"], full["suftab"][lo:hi])
        pos = full["llvtab"][:, 0]
        assert np.array_equal(d["llvtab"], full["llvtab"][(pos >= lo) & (pos < hi)])
        assert np.array_equal(d["bwtpk"], O.pack_bwt_ref(full["bwttab"][lo:hi])[0])


@pytest.mark.parametrize("kind,bases,seed,world", [("human", 30_000_000, 5, 3),
                                                   ("plant", 20_000_000, 2, 2)])
def test_range_shards_smax_with_device_stitch(kind, bases, seed, world):
    minlen = 20 if kind == "human" else 50
    text = G.synth_genome(kind, bases, seed, threads=8)
    full, (n, N, _, _) = _full(text)
    want = O.linsmax(full["lcptab"], full["llvtab"], full["bwttab"], N, minlen, threads=8)
    bnd = torch.zeros(G.BOUNDARY_BYTES * world, dtype=torch.uint8, device="cuda")
    esas, plans = [], []
    for r in range(world):
        begin = 1 + (N - 1) * r // world
        end = 1 + (N - 1) * (r + 1) // world
        e = G.DeviceEsa64(text, device=0, row_lo=begin - 1, row_hi=end + 1)
        p = e.plan(minlen, begin, end, capacity=(end - begin) // 2 + 16)
        p.run()
        p.copy_boundary(bnd.data_ptr() + G.BOUNDARY_BYTES * r)
        esas.append(e)
        plans.append(p)
    torch.cuda.synchronize()
    parts = []
    for r, p in enumerate(plans):
        p.stitch(bnd.data_ptr(), world, r)
        parts.append(p.fetch_triples())
        p.close()
    for e in esas:
        e.release()
    got = np.concatenate(parts)
    assert len(want) > 100
    assert np.array_equal(got, want), (len(got), len(want))

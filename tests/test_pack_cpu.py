"""Host packing of the BWT into the bit-plane form the scan streams
(gt_smax_pack_bwt, GT_SMAX_PK_GROUPS in include/gt_smax_hip.h) against the
numpy restatement of the layout.  Pure host code: no GPU involved."""
import numpy as np
import pytest

import genometools_smax_amd as G
import oracle_lib as O


@pytest.mark.parametrize("n", [0, 1, 15, 16, 17, 1000, 65536 + 7, 3_000_001])
def test_pack_matches_layout(n):
    rng = np.random.default_rng(n)
    bwt = rng.integers(0, 4, n, dtype=np.uint8)
    if n:
        bwt[rng.integers(0, n, max(1, n // 50))] = 254
        bwt[rng.integers(0, n, max(1, n // 70))] = 255
    got, dna = G.pack_bwt(bwt)
    want, wdna = O.pack_bwt_ref(bwt)
    assert dna and wdna
    assert np.array_equal(got, want)


def test_pack_reports_non_dna():
    bwt = np.zeros(5000, dtype=np.uint8)
    bwt[4321] = 7
    _, dna = G.pack_bwt(bwt)
    assert not dna
    bwt[4321] = 253
    assert not G.pack_bwt(bwt)[1]
    bwt[4321] = 254
    assert G.pack_bwt(bwt)[1]


def test_pack_of_reference_fixture(golden):
    e = __import__("conftest").oracle_esa("at1MB")
    got, dna = G.pack_bwt(e.bwt)
    want, _ = O.pack_bwt_ref(e.bwt)
    assert dna and np.array_equal(got, want)


@pytest.mark.parametrize("fasta", ["Atinsert.fna", "at1MB", "Random.fna", "Random-Small.fna",
                                   "TTT-small.fna"])
def test_fasta_encoding_matches_oracle(golden, fasta):
    import os
    with open(os.path.join(golden, fasta), "rb") as fh:
        buf = fh.read()
    got, ns = G.encode_fasta(buf)
    want, _ = O.encode_fasta(os.path.join(golden, fasta))
    assert np.array_equal(got, want)
    assert ns == buf.count(b">") or (ns == 1 and buf.count(b">") == 0)


def test_fasta_encoding_rejects_non_dna():
    with pytest.raises(G.SmaxError):
        G.encode_fasta(b">x\nACGTQ\n")

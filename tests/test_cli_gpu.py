"""The C host CLI (`gt repfind -smax`) end to end on the GPU."""
import os
import subprocess

import numpy as np
import pytest

import genometools_smax_amd as G
import oracle_lib as O
from conftest import GOLDEN, oracle_esa

CLI = os.path.join(G.BIN_DIR, "gt-repfind")


def _norm(lines):
    return [" ".join(l.split()) for l in lines if l.strip() and not l.startswith("#")]


def _index(tmp_path, fasta, suftab_bytes=8):
    idx = str(tmp_path / os.path.basename(fasta))
    O.index_fasta(os.path.join(GOLDEN, fasta), idx, suftab_bytes)
    return idx


@pytest.mark.gpu
@pytest.mark.parametrize("scan,width", [(False, 8), (True, 8), (True, 4)])
def test_cli_atinsert_pairs(tmp_path, scan, width):
    idx = _index(tmp_path, "Atinsert.fna", width)
    cmd = [CLI, "-smax", "-l", "8", "-ii", idx] + (["-scan"] if scan else [])
    out = subprocess.run(cmd, check=True, capture_output=True, text=True).stdout
    mine = _norm(out.splitlines())
    e = oracle_esa("Atinsert.fna")
    want = _norm(O.format_pairs(O.smax_pairs(O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, 8),
                                             e.suftab), e.separators))
    assert mine == want
    assert len(mine) == 205
    with open(os.path.join(GOLDEN, "repfind-8-Atinsert.txt")) as fh:
        assert set(mine) <= set(_norm(fh))


@pytest.mark.gpu
@pytest.mark.parametrize("scan,width", [(False, 8), (True, 4)])
def test_cli_maxpairs_matches_reference_golden(tmp_path, scan, width):
    # `gt repfind -l 8 -ii Atinsert` (default -f: maximal pairs) == the
    # reference's testdata/repfind-8-Atinsert.txt line for line, in order (the
    # reference's own test diffs it: testsuite/gt_idxsearch_include.rb:149-151)
    idx = _index(tmp_path, "Atinsert.fna", width)
    out = subprocess.run([CLI, "-l", "8", "-ii", idx] + (["-scan"] if scan else []), check=True,
                         capture_output=True, text=True).stdout
    with open(os.path.join(GOLDEN, "repfind-8-Atinsert.txt")) as fh:
        want = _norm(fh)
    mine = _norm(out.splitlines())
    assert len(mine) == 452 and mine == want


@pytest.mark.gpu
def test_cli_at1mb_intervals_and_gpus(tmp_path):
    idx = _index(tmp_path, "at1MB")
    e = oracle_esa("at1MB")
    want = O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials, 20)
    for gpus in ("1", "4"):
        out = subprocess.run([CLI, "-smax", "-l", "20", "-ii", idx, "-intervals", "-gpus", gpus],
                             check=True, capture_output=True, text=True).stdout
        got = np.array([[int(x) for x in l.split()] for l in out.splitlines()], dtype=np.uint64)
        assert np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("args", [["-smax", "-l", "20"], ["-smax", "-l", "20", "-gpus", "3"],
                                  ["-l", "20"], ["-l", "30", "-scan"]])
def test_cli_gpu_lines_equal_host_lines(tmp_path, args):
    # F4: the GPU-formatted output is byte-identical to the host printf path
    idx = _index(tmp_path, "at1MB")
    gpu = subprocess.run([CLI, "-ii", idx] + args, check=True, capture_output=True).stdout
    host = subprocess.run([CLI, "-ii", idx, "-hostformat"] + args, check=True,
                          capture_output=True).stdout
    assert len(gpu) > 10000 and gpu == host


def _many_seqs_fasta(path, rng, nseq):
    with open(path, "w") as fh:
        for k in range(nseq):
            n = int(rng.integers(1, 400))
            s = "".join("ACGT"[c] for c in rng.integers(0, 4, n))
            if k % 7 == 0:
                s = "ACGTTGCAAGGCTTAACCGGTTA" * 3 + s     # shared repeat across sequences
            fh.write(">s%d\n%s\n" % (k, s))


@pytest.mark.gpu
def test_cli_many_sequences_lines(tmp_path):
    # thousands of sequences: multi-digit seqnums and relpos through the GPU
    # formatter, against the oracle's restatement of the output function
    fasta = str(tmp_path / "many.fna")
    _many_seqs_fasta(fasta, np.random.default_rng(5), 3000)
    idx = str(tmp_path / "many")
    O.index_fasta(fasta, idx, 8)
    e = O.Esa(G.encode_fasta(open(fasta, "rb").read())[0])
    for args, want in ((["-smax", "-l", "12"],
                        O.format_pairs(O.smax_pairs(O.linsmax(e.lcpbytes, e.llv, e.bwt, e.nonspecials,
                                                              12), e.suftab), e.separators)),
                       (["-l", "12"], O.format_pairs(O.maxpairs(e, 12), e.separators))):
        out = subprocess.run([CLI, "-ii", idx] + args, check=True, capture_output=True,
                             text=True).stdout
        assert len(want) > 1000
        assert out.splitlines() == [w.rstrip("\n") for w in want]


def test_cli_errors(tmp_path):
    r = subprocess.run([CLI, "-l", "8", "-ii", "x"], capture_output=True, text=True)
    assert r.returncode == 1 and "gt repfind: error:" in r.stderr
    r = subprocess.run([CLI, "-smax", "-r", "-ii", "x"], capture_output=True, text=True)
    assert r.returncode == 1 and "exclude each other" in r.stderr
    r = subprocess.run([CLI, "-l", "8", "-r", "-ii", "x"], capture_output=True, text=True)
    assert r.returncode == 1 and "not part of this build" in r.stderr
    r = subprocess.run([CLI, "-intervals", "-ii", "x"], capture_output=True, text=True)
    assert r.returncode == 1 and "requires option" in r.stderr
    r = subprocess.run([CLI, "-smax", "-l", "0", "-ii", "x"], capture_output=True, text=True)
    assert r.returncode == 1
    r = subprocess.run([CLI, "-smax", "-ii", str(tmp_path / "missing")], capture_output=True, text=True)
    assert r.returncode == 1 and "cannot open" in r.stderr
    idx = _index(tmp_path, "Atinsert.fna", 4)
    r = subprocess.run([CLI, "-smax", "-ii", idx], capture_output=True, text=True)
    assert r.returncode == 1 and "number of mapped units" in r.stderr


SFXMAP = os.path.join(G.BIN_DIR, "gt-sfxmap")


@pytest.mark.gpu
@pytest.mark.parametrize("fasta", ["Reads2.fna", "Atinsert.fna", "at1MB"])
def test_sfxmap_enumlcpitvtree_bu(tmp_path, fasta):
    # `gt dev sfxmap -enumlcpitvtreeBU -esa IDX`: the lcpitvs visitor's
    # L/B lines (src/match/esa_lcpintervals_visitor.c:30-61), in the order of
    # gt_esa_bottomup, from the GPU tree
    idx = _index(tmp_path, fasta)
    out = subprocess.run([SFXMAP, "-enumlcpitvtreeBU", "-esa", idx], check=True,
                         capture_output=True, text=True).stdout.splitlines()
    ev = O.bottomup_events(oracle_esa(fasta))
    want = []
    for r in ev:
        if r[0] == 0:
            want.append("L %d %d %d %d" % (r[1], r[2], r[3], r[4]))
        elif r[0] == 1:
            want.append("B %d %d %d %d %d" % (r[1], r[2], r[3], r[4], r[5]))
    assert out == want
    # the reference's check: the BU lines equal the depth-first traversal's
    # (-enumlcpitvtree, gt_depthfirstesa), restated in the oracle
    dfs = O.dfs_events(oracle_esa(fasta))
    assert out == ["L %d %d %d %d" % tuple(r[1:5]) if r[0] == 0 else
                   "B %d %d %d %d %d" % tuple(r[1:6]) for r in dfs]


def test_sfxmap_errors():
    r = subprocess.run([SFXMAP, "-esa", "x"], capture_output=True, text=True)
    assert r.returncode == 1 and "gt sfxmap: error:" in r.stderr
    r = subprocess.run([SFXMAP, "-enumlcpitvtreeBU"], capture_output=True, text=True)
    assert r.returncode == 1 and "mandatory" in r.stderr

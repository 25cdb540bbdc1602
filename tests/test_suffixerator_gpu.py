"""The GPU suffixerator CLI (`bin/gt-suffixerator`):
FASTA -> GPU-built suffix array -> .suf/.lcp/.llv/.bwt/.prj files.

  - byte-identical files to the oracle's suffixerator restatement (which
    reproduces the reference's .prj fixtures and repfind golden) for the
    reference's FASTA fixtures, with 8- and 4-byte .suf;
  - `gt-repfind -smax` on a GPU-built index of BASELINE config C2 (100 Mbp
    uniform ACGT, seed 42) prints the oracle's intervals, and the written
    tables equal the 32-bit GPU builder's in memory.
"""
import filecmp
import os
import subprocess

import numpy as np
import pytest

import genometools_smax_amd as G
import oracle_lib as O
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

SFX = os.path.join(G.BIN_DIR, "gt-suffixerator")
REPFIND = os.path.join(G.BIN_DIR, "gt-repfind")


@pytest.mark.parametrize("fasta", ["Atinsert.fna", "at1MB", "Random.fna", "TTT-small.fna"])
@pytest.mark.parametrize("width", [8, 4])
def test_files_equal_oracle(tmp_path, fasta, width):
    db = os.path.join(GOLDEN, fasta)
    gpu = str(tmp_path / "gpu")
    orc = str(tmp_path / "orc")
    cmd = [SFX, "-db", db, "-indexname", gpu, "-dna", "-suf", "-lcp", "-bwt"]
    subprocess.run(cmd + (["-suftabuint"] if width == 4 else []), check=True)
    O.index_fasta(db, orc, width)
    for suffix in (".suf", ".lcp", ".llv", ".bwt", ".prj"):
        assert filecmp.cmp(gpu + suffix, orc + suffix, shallow=False), suffix


def test_cli_errors(tmp_path):
    bad = tmp_path / "bad.fna"
    bad.write_text(">x\nACGTXACGT\n")
    r = subprocess.run([SFX, "-db", str(bad), "-indexname", str(tmp_path / "i")], capture_output=True,
                       text=True)
    assert r.returncode == 1 and r.stderr.startswith("gt suffixerator: error:")
    r = subprocess.run([SFX, "-indexname", "x"], capture_output=True, text=True)
    assert r.returncode == 1 and "-db" in r.stderr


def _write_fasta(path, text):
    """Encoded text (0..3, 254, 255 separators) -> FASTA lines."""
    alpha = np.frombuffer(b"ACGT", dtype=np.uint8)
    seqs = np.split(text, np.flatnonzero(text == 255))
    with open(path, "wb") as fh:
        for k, s in enumerate(seqs):
            s = s[s != 255]
            fh.write(b">seq%d\n" % k)
            chars = np.where(s == 254, ord("N"), alpha[np.minimum(s, 3)]).astype(np.uint8)
            for i in range(0, len(chars), 1 << 20):
                fh.write(chars[i:i + (1 << 20)].tobytes())
            fh.write(b"\n")


def test_c2_gpu_index_through_repfind(tmp_path):
    text = G.synth_genome("uniform", 100_000_000, 42, threads=16)
    fasta = str(tmp_path / "c2.fna")
    _write_fasta(fasta, text)
    idx = str(tmp_path / "c2")
    subprocess.run([SFX, "-db", fasta, "-indexname", idx, "-v"], check=True, capture_output=True)
    # the files against the in-memory 32-bit GPU builder
    esa = G.DeviceEsa(text, device=0, keep_suftab=True)
    want = esa.download(suftab=True)
    esa.release()
    assert np.array_equal(np.fromfile(idx + ".lcp", dtype=np.uint8), want["lcptab"])
    assert np.array_equal(np.fromfile(idx + ".bwt", dtype=np.uint8), want["bwttab"])
    assert np.array_equal(np.fromfile(idx + ".suf", dtype=np.uint64), want["suftab"])
    llv = np.fromfile(idx + ".llv", dtype=np.uint64).reshape(-1, 2)
    assert np.array_equal(llv, want["llvtab"])
    # gt repfind -smax on the GPU-built index
    out = subprocess.run([REPFIND, "-smax", "-l", "20", "-ii", idx, "-intervals"], check=True,
                         capture_output=True, text=True).stdout
    got = np.array([[int(x) for x in l.split()] for l in out.splitlines() if l and l[0] != "#"],
                   dtype=np.uint64).reshape(-1, 3)
    N = len(text) - int(np.count_nonzero(text >= 254))
    ref = O.linsmax(want["lcptab"], want["llvtab"], want["bwttab"], N, 20, threads=8)
    assert len(ref) > 1000
    assert np.array_equal(got, ref)

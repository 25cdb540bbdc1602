#!/usr/bin/env python3
"""F4 timing: `gt-repfind` with pair lines formatted on the GPU (default)
vs the host printf path (-hostformat), output to /dev/null, on a GPU-built
index (bin/gt-suffixerator) of a synthetic genome.  Prints one JSON line per
mode: wall seconds of the whole CLI run (index mapping included) and lines."""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import genometools_smax_amd as G  # noqa: E402


def write_fasta(path, text):
    alpha = np.frombuffer(b"ACGT", dtype=np.uint8)
    with open(path, "wb") as fh:
        for k, s in enumerate(np.split(text, np.flatnonzero(text == 255))):
            s = s[s != 255]
            fh.write(b">seq%d\n" % k)
            fh.write(np.where(s == 254, ord("N"), alpha[np.minimum(s, 3)]).astype(np.uint8).tobytes())
            fh.write(b"\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="human")
    ap.add_argument("--bases", type=int, default=20_000_000)
    ap.add_argument("--minlen", type=int, default=100)
    args = ap.parse_args()
    d = tempfile.mkdtemp(prefix="lines")
    fa, idx = os.path.join(d, "g.fna"), os.path.join(d, "g")
    write_fasta(fa, G.synth_genome(args.kind, args.bases, 1))
    subprocess.run([os.path.join(G.BIN_DIR, "gt-suffixerator"), "-db", fa, "-indexname", idx],
                   check=True)
    cli = os.path.join(G.BIN_DIR, "gt-repfind")
    for mode in ("-smax", "-f"):
        for fmt in ([], ["-hostformat"]):
            cmd = [cli, "-l", str(args.minlen), "-ii", idx, "-v"] + ([mode] if mode == "-smax" else []) + fmt
            t0 = time.perf_counter()
            r = subprocess.run(cmd, check=True, capture_output=True)
            el = time.perf_counter() - t0
            nlines = r.stdout.count(b"\n") - 2
            print(json.dumps({"mode": mode, "format": "host" if fmt else "gpu", "seconds": round(el, 3),
                              "lines": nlines, "bytes": len(r.stdout),
                              "workload": "%d bp %s, minlen %d" % (args.bases, args.kind, args.minlen)}),
                  flush=True)


if __name__ == "__main__":
    main()

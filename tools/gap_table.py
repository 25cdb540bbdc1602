#!/usr/bin/env python3
"""Diagnostic: per-kernel start/end of the last smax steps in a rocprofv3
kernel-trace database (gaps between the step's kernels)."""
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
rows = con.execute("select name, start, end, grid_x, queue_id from kernels order by start").fetchall()
rows = [r for r in rows if "smax" in r[0] or "scan_config" in r[0]][-n:]
t0 = rows[0][1]
for r in rows:
    print("%-28s %10.1f %10.1f dur %8.1f grid %8d q %d"
          % (r[0][:28], (r[1] - t0) / 1e3, (r[2] - t0) / 1e3, (r[2] - r[1]) / 1e3, r[3], r[4]))

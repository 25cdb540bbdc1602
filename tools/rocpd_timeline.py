#!/usr/bin/env python3
"""Kernel timeline of the last K launches in a rocprofv3 rocpd database:
name, duration and the gap before each launch (us).  Args: DB [K]."""
import sqlite3
import sys

db = sys.argv[1]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 40
con = sqlite3.connect(db)
objs = [r[0] for r in con.execute("select name from sqlite_master where type in ('table','view')")]
src = None
for name in objs:
    if "kernel" not in name.lower():
        continue
    cols = [r[1] for r in con.execute("pragma table_info('%s')" % name)]
    if "start" in cols and "end" in cols and ("name" in cols or "kernel_name" in cols):
        src = (name, "name" if "name" in cols else "kernel_name")
        break
if src is None:
    print("no kernel view among:", objs)
    sys.exit(1)
rows = con.execute("select %s, start, end from %s order by start" % (src[1], src[0])).fetchall()
rows = rows[-k:]
prev_end = None
for name, st, en in rows:
    short = name.split("(")[0]
    if "rocprim" in short:
        short = "rocprim"
    gap = (st - prev_end) / 1000.0 if prev_end is not None else 0.0
    print("%-34s dur %8.1f us  gap %7.1f us" % (short[:34], (en - st) / 1000.0, gap))
    prev_end = max(prev_end or en, en)

#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counters per (kernel, dispatch) from rocpd databases
and print one row per counter (values of the last dispatch of KERNEL)."""
import sqlite3
import sys

kernel = sys.argv[1]
vals = {}
for db in sys.argv[2:]:
    con = sqlite3.connect(db)
    rows = con.execute("select dispatch_id, counter_name, sum(value), max(duration) from "
                       "counters_collection where kernel_name like ? group by dispatch_id, "
                       "counter_name order by dispatch_id", ("%" + kernel + "%",)).fetchall()
    for d, name, v, dur in rows:
        vals[name] = (v, dur)
for k in sorted(vals):
    v, dur = vals[k]
    print("%-28s %18.0f   (dispatch %.3f ms)" % (k, v, dur / 1e6))

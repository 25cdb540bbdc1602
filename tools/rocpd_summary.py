#!/usr/bin/env python3
"""Turn rocprofv3 rocpd databases into the summaries committed under
profiles/.

  rocpd_summary.py stats  DB OUT.csv                   kernel-trace --stats table
  rocpd_summary.py pmc    OUT.json KERNEL CONFIG DB... per-launch counters of KERNEL
  rocpd_summary.py pmcall OUT.json CONFIG DB...        per-launch HBM bytes of every kernel

`pmc` keeps every counter of the passes (per launch), the HBM bytes when
FETCH_SIZE and WRITE_SIZE are among them, the bench config the passes ran
(tools/k1_once.py CONFIG) and the build identity of the library they ran on
(gt_smax_build_id): bench.py uses a profile's traffic only when both match
the run it reports.

For `pmc`, each DB is one `rocprofv3 --pmc <COUNTER>` pass (FETCH_SIZE and
WRITE_SIZE do not fit one pass on gfx950).  FETCH_SIZE / WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE counts half the bytes of wide streaming reads
(/opt/skills/guides/MI355X_MICROARCH.md, HBM section), so read bytes =
2 x 1024 x FETCH_SIZE; write bytes = 1024 x WRITE_SIZE.
"""
import csv
import json
import sqlite3
import sys


def stats(db, out):
    con = sqlite3.connect(db)
    rows = con.execute("select name, total_calls, total_duration, average, percentage "
                       "from top_kernels").fetchall()
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "calls", "total_us", "average_us", "percent"])
        for name, calls, tot, avg, pct in rows:
            short = name.replace("(anonymous namespace)::", "")
            if "rocprim" in short:
                # rocprim trampoline: keep the wrapped algorithm's config name
                key = short.split("wrapped_")[1].split("<")[0] if "wrapped_" in short else "kernel"
                short = "rocprim::" + key
            else:
                short = short.split("(")[0]
            w.writerow([short, calls, "%.0f" % tot, "%.1f" % avg, "%.2f" % pct])
    print("wrote", out, len(rows), "kernels")


def pmc(out, kernel, config, dbs):
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import genometools_smax_amd as G
    res = {"kernel": kernel, "config": config, "build_id": G.build_id(), "passes": {}}
    for db in dbs:
        con = sqlite3.connect(db)
        rows = con.execute("select counter_name, value, duration from counters_collection "
                           "where kernel_name like ?", ("%" + kernel + "%",)).fetchall()
        for name, value, dur in rows:
            res["passes"].setdefault(name, []).append(float(value))
    fetch = res["passes"].get("FETCH_SIZE", [])
    write = res["passes"].get("WRITE_SIZE", [])
    if fetch:
        res["fetch_kib_per_launch"] = sum(fetch) / len(fetch)
        res["read_bytes_per_launch"] = 2 * 1024 * res["fetch_kib_per_launch"]
    if write:
        res["write_kib_per_launch"] = sum(write) / len(write)
        res["write_bytes_per_launch"] = 1024 * res["write_kib_per_launch"]
    if fetch and write:
        res["hbm_bytes_per_launch"] = res["read_bytes_per_launch"] + res["write_bytes_per_launch"]
        res["method"] = ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                         "read = 2 x 1024 x FETCH_SIZE (gfx950 half-count correction), "
                         "write = 1024 x WRITE_SIZE")
    res["per_launch"] = {k: sum(v) / len(v) for k, v in res["passes"].items() if v}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "passes"}, indent=1))


def pmcall(out, config, dbs):
    """FETCH_SIZE / WRITE_SIZE per launch of every kernel in the passes
    (same corrections as pmc), keyed by the short kernel name."""
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import genometools_smax_amd as G
    per = {}
    for db in dbs:
        con = sqlite3.connect(db)
        rows = con.execute("select kernel_name, counter_name, dispatch_id, sum(value), max(duration) "
                           "from counters_collection group by kernel_name, counter_name, dispatch_id"
                           ).fetchall()
        for name, cname, _d, value, dur in rows:
            short = name.replace("(anonymous namespace)::", "").split("(")[0]
            k = per.setdefault(short, {}).setdefault(cname, [])
            k.append((float(value), float(dur or 0)))
    res = {"config": config, "build_id": G.build_id(),
           "method": ("rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                      "read = 2 x 1024 x FETCH_SIZE (gfx950 half-count correction), "
                      "write = 1024 x WRITE_SIZE; per launch = mean over the kernel's launches"),
           "kernels": {}}
    for short, cs in sorted(per.items()):
        d = {}
        if "FETCH_SIZE" in cs:
            v = cs["FETCH_SIZE"]
            d["launches"] = len(v)
            d["read_bytes_per_launch"] = 2 * 1024 * sum(x for x, _ in v) / len(v)
        if "WRITE_SIZE" in cs:
            v = cs["WRITE_SIZE"]
            d["write_bytes_per_launch"] = 1024 * sum(x for x, _ in v) / len(v)
        if "read_bytes_per_launch" in d and "write_bytes_per_launch" in d:
            d["hbm_bytes_per_launch"] = d["read_bytes_per_launch"] + d["write_bytes_per_launch"]
        for cname, v in cs.items():            # every other counter, per launch
            if cname not in ("FETCH_SIZE", "WRITE_SIZE"):
                d[cname] = sum(x for x, _ in v) / len(v)
        res["kernels"][short] = d
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    for k, d in res["kernels"].items():
        print("%-50s %s" % (k[:50], {x: round(y) for x, y in d.items()}))


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        stats(sys.argv[2], sys.argv[3])
    elif sys.argv[1] == "pmcall":
        pmcall(sys.argv[2], sys.argv[3], sys.argv[4:])
    else:
        pmc(sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[5:])

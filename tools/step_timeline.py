#!/usr/bin/env python3
"""Diagnostic: where a plan step's time goes between kernels.  Reads the
kernel trace CSV of `rocprofv3 --kernel-trace --output-format csv` over a
run of repeated plan steps (K1 -> K1b -> K3 on one stream) and prints, per
kernel, the median duration and the median gap from the previous kernel's
end to its start, plus the median step (K1 start to the next K1 start).

  step_timeline.py TRACE_DIR_OR_CSV [FIRST_KERNEL_REGEX]"""
import csv
import glob
import os
import re
import statistics
import sys

src = sys.argv[1]
first = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"smax_scan_kernel")
if os.path.isdir(src):
    found = glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True)
    if not found:
        sys.exit("no *kernel_trace.csv under %s" % src)
    src = found[0]
rows = []
with open(src) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
short = lambda n: re.sub(r"\(.*$", "", n).replace("void ", "").strip()
# group into steps: a step starts at each launch of the first kernel
steps, cur = [], None
for s, e, n in rows:
    n = short(n)
    if first.search(n):
        if cur:
            steps.append(cur)
        cur = []
    if cur is not None:
        cur.append((s, e, n))
if cur:
    steps.append(cur)
steps = steps[len(steps) // 4:]        # drop the warm-up quarter
if len(steps) < 3:
    sys.exit("too few steps (%d)" % len(steps))
dur, gap = {}, {}
for st in steps:
    prev_end = None
    for s, e, n in st:
        dur.setdefault(n, []).append((e - s) / 1e3)
        if prev_end is not None:
            gap.setdefault(n, []).append((s - prev_end) / 1e3)
        prev_end = e
period = [(b[0][0] - a[0][0]) / 1e3 for a, b in zip(steps, steps[1:])]
busy = [(st[-1][1] - st[0][0]) / 1e3 for st in steps]
print("%d steps from %s" % (len(steps), os.path.basename(src)))
print("median step period %.2f us, first kernel start -> last kernel end %.2f us" %
      (statistics.median(period), statistics.median(busy)))
for n in dur:
    g = gap.get(n)
    print("  %-40s dur %8.2f us  gap before %s" %
          (n[:40], statistics.median(dur[n]),
           "%6.2f us" % statistics.median(g) if g else "   -"))

#!/usr/bin/env python3
"""Reduce tools/calib_masked.sh's output (tools/membw_masked.hip under
rocprofv3): per variant the kernel time, the 128-B lines and 64-B segments of
the masked column that hold a selected row (counted by the kernel itself),
and FETCH_SIZE x 2 (gfx950) / TCC_EA0_RDREQ x 128 B per row -- which byte
count the counters agree with. usage: membw_masked.py <calib dir>"""
import collections
import csv
import os
import re
import sys

d = sys.argv[1]
rows = 1e9
table = {}
for ln in open(os.path.join(d, "table.txt")):
    m = re.match(r"(stream|tile) p=(\d+)/1000\s+([\d.]+) ms\s+seg64/row ([\d.]+) seg128/row ([\d.]+)", ln)
    if m:
        table[(m.group(1), int(m.group(2)))] = (float(m.group(3)), float(m.group(4)), float(m.group(5)))
    m = re.match(r"rows (\d+)", ln)
    if m:
        rows = float(m.group(1))


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        per[(r["Dispatch_Id"], r["Kernel_Name"])] += float(r["Counter_Value"])
    for (_, k), v in per.items():
        m = re.match(r"void masked_(stream|tile)<(\d+)>", k)
        if m:
            acc[(m.group(1), int(m.group(2)))].append(v)
    return {k: sum(v) / len(v) for k, v in acc.items()}


fetch = per_kernel(os.path.join(d, "fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
rdreq = per_kernel(os.path.join(d, "rdreq", "rdreq_counter_collection.csv"), "TCC_EA0_RDREQ_sum")
print("rows per launch %.0f; column a read by every row (8 B/row), column c only where selected" % rows)
print("%-8s %6s %9s %10s %11s %11s %12s %12s %9s" % ("variant", "p", "ms", "lines128", "B/row@64B", "B/row@128B",
                                                     "FETCHx2 B/r", "RDREQx128", "GB/s@128"))
for k in sorted(table):
    ms, s64, s128 = table[k]
    b64 = 8 + 64 * s64
    b128 = 8 + 128 * s128
    f = fetch.get(k, float("nan")) * 1024 * 2 / rows
    q = rdreq.get(k, float("nan")) * 128 / rows
    print("%-8s %6.3f %9.4f %10.5f %11.4f %11.4f %12.4f %12.4f %9.1f" % (k[0], k[1] / 1000, ms, s128, b64, b128, f, q,
                                                                       b128 * rows / ms / 1e6))
print("tile: pass 2 re-reads a's lines of the selected rows; those re-reads appear as extra requests")

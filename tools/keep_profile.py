#!/usr/bin/env python3
"""Copy a tools/profile_r04.sh output directory into profiles/<round>/: per
run the bench lines, traffic.json, the rocprofv3 kernel stats, and the
kernel trace / PMC rows of the launches over at least 1M work items (the
1024-row batch lines dispatch tens of thousands of small kernels, which the
stats file already summarises).
usage: tools/keep_profile.py gpurun_out/r04 profiles/r04"""
import csv
import os
import shutil
import sys

MIN_GRID = 1 << 20


def filtered(src, dst, grid_col):
    with open(src, newline="") as f, open(dst, "w", newline="") as g:
        r = csv.reader(f)
        w = csv.writer(g, quoting=csv.QUOTE_NONNUMERIC)
        head = next(r)
        w.writerow(head)
        gi = [head.index(c) for c in grid_col]
        for row in r:
            n = 1
            for i in gi:
                n *= int(float(row[i]))
            if n >= MIN_GRID:
                w.writerow(row)


def main(src, dst):
    for run in sorted(os.listdir(src)):
        s, d = os.path.join(src, run), os.path.join(dst, run)
        if not os.path.isdir(s):
            continue
        os.makedirs(d, exist_ok=True)
        for f in ("bench.json", "fetch_bench.json", "write_bench.json", "traffic.json", "box.txt"):
            if os.path.exists(os.path.join(s, f)):
                shutil.copy(os.path.join(s, f), os.path.join(d, f))
        shutil.copy(os.path.join(s, "kt", "kt_kernel_stats.csv"), os.path.join(d, "kernel_stats.csv"))
        filtered(os.path.join(s, "kt", "kt_kernel_trace.csv"), os.path.join(d, "kernel_trace.csv"),
                 ["Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"])
        for p in ("fetch", "write"):
            filtered(os.path.join(s, p, "%s_counter_collection.csv" % p), os.path.join(d, "%s_counter_collection.csv" % p),
                     ["Grid_Size"])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])

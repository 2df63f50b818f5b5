#!/usr/bin/env python3
"""Per-dispatch summary of a rocprofv3 --pmc counter_collection.csv: counters
summed over instances, per-wave figures for the filter kernels.
usage: tools/pmc_summary.py counter_collection.csv [min_waves]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    min_waves = float(sys.argv[2]) if len(sys.argv) > 2 else 0
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        if "dfmi_" not in r["Kernel_Name"]:
            continue
        agg[(int(r["Dispatch_Id"]), r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for (d, k), c in sorted(agg.items()):
        w = c.get("SQ_WAVES", 0)
        if w and w < min_waves:
            continue
        per = {n: (v / w if w and n.startswith("SQ_INSTS") else v) for n, v in sorted(c.items())}
        print(d, k, " ".join("%s=%.4g" % (n, v) for n, v in per.items()))


if __name__ == "__main__":
    main()

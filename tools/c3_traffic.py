#!/usr/bin/env python3
"""HBM traffic of the two C3 queries from tools/c3_counters.sh's passes.

tools/c3_probe.py with the default variant launches each query 8 times on one
1.25e8-row batch (equality first, then the gather); the first launch of each
is excluded (compile / first touch). Bytes per MI355X_MICROARCH.md's gfx950
corrections: read = 2 x FETCH_SIZE KiB x 1024, write = WRITE_SIZE KiB x 1024.

usage: tools/c3_traffic.py <gpurun_out/tag> <out.json>
"""
import csv
import json
import sys

ROWS = 125_000_000
PER_QUERY = 8


def launches(path, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Kernel_Name"] == "dfmi_query" and r["Counter_Name"] == counter:
            vals[int(r["Dispatch_Id"])] = vals.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def durations(path):
    d = [(int(r["Dispatch_Id"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
         for r in csv.DictReader(open(path)) if r["Kernel_Name"] == "dfmi_query"]
    return [ms for _, ms in sorted(d)]


def main():
    d, out = sys.argv[1], sys.argv[2]
    fetch = launches(d + "/fetch/fetch_counter_collection.csv", "FETCH_SIZE")
    write = launches(d + "/write/write_counter_collection.csv", "WRITE_SIZE")
    kt = durations(d + "/kt/kt_kernel_trace.csv")
    assert len(fetch) == len(write) == len(kt) == 2 * PER_QUERY, (len(fetch), len(write), len(kt))
    # algorithmic bytes per row, from the probe's own line (bench.py's C3 formula)
    alg = {}
    for part in open(d + "/kt_probe.log").read().split("|")[1:]:
        f = part.split()
        qn, ms, frac = f[0], float(f[1]), float(f[4])
        alg[qn] = frac * 8e12 * ms * 1e-3 / ROWS
    res = {}
    for i, qn in enumerate(("eq", "lt")):
        sl = slice(i * PER_QUERY + 1, (i + 1) * PER_QUERY)
        rd = 2 * 1024 * sum(fetch[sl]) / (PER_QUERY - 1)
        wr = 1024 * sum(write[sl]) / (PER_QUERY - 1)
        ms = sum(kt[sl]) / (PER_QUERY - 1)
        res[qn] = {"rows": ROWS, "launches_averaged": PER_QUERY - 1, "read_bytes": rd, "write_bytes": wr,
                   "traffic_bytes": rd + wr, "traffic_bytes_per_row": round((rd + wr) / ROWS, 2),
                   "algorithmic_bytes_per_row": round(alg[qn], 3), "kernel_ms_rocprof": round(ms, 4),
                   "traffic_gbs": round((rd + wr) / (ms * 1e-3) / 1e9, 1),
                   "algorithmic_gbs": round(alg[qn] * ROWS / (ms * 1e-3) / 1e9, 1)}
    res["note"] = ("tools/c3_counters.sh + tools/c3_traffic.py: one 1.25e8-row C3 batch, %d launches per query "
                   "(first excluded); read = 2 x FETCH_SIZE KiB x 1024 (gfx950), write = WRITE_SIZE KiB x 1024"
                   % PER_QUERY)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

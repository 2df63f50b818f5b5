#!/usr/bin/env python3
"""Per-kernel table of a profiled bench run (tools/profile_r03.sh): for every
(kernel name, grid size) the launch count and average duration from the
rocprofv3 kernel trace, the kernel's resources (VGPRs, SGPRs, scratch, LDS),
and its HBM traffic per launch from the separate FETCH_SIZE / WRITE_SIZE PMC
passes, corrected as MI355X_MICROARCH.md "HBM" prescribes: FETCH_SIZE and
WRITE_SIZE are KiB; on gfx950 FETCH_SIZE tallies 128-byte read requests at
64 bytes, so it is doubled. Calibrated (tools/membw_masked.hip,
profiles/r06/calib_masked/summary.txt) for 8-byte streaming loads and for
lane-masked 8-byte loads: FETCH_SIZE x 2 = 128 B x the 128-byte lines that
hold a loaded row, exactly; a line loaded again after it left the L2 counts
again (Infinity-Cache hits included), so these are memory-side request
bytes, an upper bound on HBM bytes. Query kernels are named per shape
(dfmi_<filter|project|agg>_<hash>, jit.cpp), so every bench line's kernel has
its own row. Writes <dir>/traffic.json, which bench.py reads to report
roofline.traffic next to the formula bytes.

usage: tools/traffic.py <profile dir with kt/ fetch/ write/ subdirs>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _find(d, pattern):
    hits = sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))
    return hits[0] if hits else None


def kernel_trace(path):
    """(name, grid) -> launches, mean duration (ns), resources."""
    out = {}
    acc = defaultdict(list)
    meta = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        acc[(name, grid)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        meta[(name, grid)] = {"vgpr": int(r["VGPR_Count"]), "agpr": int(r["Accum_VGPR_Count"]),
                              "sgpr": int(r["SGPR_Count"]), "scratch": int(r["Scratch_Size"]),
                              "lds": int(r["LDS_Block_Size"]), "block": int(r["Workgroup_Size_X"])}
    for k, v in acc.items():
        out[k] = {"launches": len(v), "avg_ns": sum(v) / len(v), "min_ns": min(v), "max_ns": max(v), **meta[k]}
    return out


def counter(path, name):
    """(kernel name, grid) -> mean counter value per launch."""
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != name:
            continue
        acc[(r["Kernel_Name"], int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main():
    d = sys.argv[1]
    kt = kernel_trace(_find(os.path.join(d, "kt"), "*kernel_trace.csv"))
    fp = _find(os.path.join(d, "fetch"), "*counter_collection.csv")
    wp = _find(os.path.join(d, "write"), "*counter_collection.csv")
    fetch = counter(fp, "FETCH_SIZE") if fp else {}
    write = counter(wp, "WRITE_SIZE") if wp else {}
    kernels = []
    for (name, grid), t in sorted(kt.items(), key=lambda x: -x[1]["avg_ns"] * x[1]["launches"]):
        if not name.startswith("dfmi_"):
            continue
        e = {"kernel": name, "grid": grid, **t}
        if (name, grid) in fetch and (name, grid) in write:
            f, nf = fetch[(name, grid)]
            w, nw = write[(name, grid)]
            e.update({"pmc_launches": [nf, nw], "fetch_size_kib": f, "write_size_kib": w,
                      "read_bytes": f * 1024 * 2, "write_bytes": w * 1024,
                      "traffic_bytes": f * 1024 * 2 + w * 1024,
                      "read_correction": "2 x FETCH_SIZE x 1024"})
            e["traffic_gbs_at_avg"] = round(e["traffic_bytes"] / e["avg_ns"], 1)
        kernels.append(e)
    box = None  # the box the profile ran on (tools/profile_r05.sh writes it): bench lines name theirs too
    if os.path.exists(os.path.join(d, "box.txt")):
        box = open(os.path.join(d, "box.txt")).read().strip()
        for e in kernels:
            e["box"] = box
    out = {"source": d, "box": box, "kernels": kernels,
           "note": "avg_ns from the kernel trace of the same bench command; traffic per launch from separate "
                   "FETCH_SIZE / WRITE_SIZE passes of it"}
    json.dump(out, open(os.path.join(d, "traffic.json"), "w"), indent=1)
    for e in kernels:
        print("%-28s grid %11d  x%-4d %9.1f us  vgpr %3d scratch %4d  traffic %s" % (
            e["kernel"][:28], e["grid"], e["launches"], e["avg_ns"] / 1e3, e["vgpr"], e["scratch"],
            "%.3g B" % e["traffic_bytes"] if "traffic_bytes" in e else "-"))


if __name__ == "__main__":
    main()

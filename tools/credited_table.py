#!/usr/bin/env python3
"""Every bench line of a profile (profiles/<round>/<run>/bench.json) with
bench.py's roofline() recomputed against the same profile's traffic.json:
HIP-event ms, rocprof ms, formula, moved-bytes and PMC fractions, `frac` -- the lowest
(DESIGN.md §6). usage: tools/credited_table.py [runs...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def lines(d):
    out = []

    def walk(o, path):
        if isinstance(o, dict):
            if isinstance(o.get("roofline"), dict) and "kernel" in o["roofline"]:
                out.append((path, o["roofline"]))
            for k, v in o.items():
                if k != "roofline":
                    walk(v, path + "/" + k)
    walk(d, "")
    return out


def main(runs):
    seen = set()
    for run in runs:
        b = json.load(open(os.path.join(bench.PROFILE_DIR, run, "bench.json")))
        for path, r in lines(b):
            if (r["kernel"], run) in seen or path.startswith("/sweep"):
                continue
            seen.add((r["kernel"], run))
            L = r.get("launches_per_step", 1)
            alg = r["achieved"] * 1e9 * r["kernel_ms"] * 1e-3
            rows = alg * L / r["algorithmic_bytes_per_row"]
            moved = r["moved_bytes_per_row"] * rows / L if "moved_bytes_per_row" in r else None
            n = bench.roofline(r["kernel"], alg, r["kernel_ms"], rows, launches=L, run=run, moved=moved)
            rp = n.get("rocprof", {}).get("avg_ms", float("nan"))
            print("%-9s %-14s %-22s hip %.4f rocprof %.4f (%+.1f%%) | formula %.2f B/row -> %.3f | moved %s | PMC %.2f B/row"
                  " %.0f GB/s -> %.3f | frac %.3f (%s)%s" % (
                      run, path or "/", r["kernel"], r["kernel_ms"], rp, (r["kernel_ms"] / rp - 1) * 100,
                      n["algorithmic_bytes_per_row"], n["formula_frac"],
                      "%.2f B/row -> %.3f" % (n["moved_bytes_per_row"], n["moved_frac"]) if moved is not None else "-",
                      n.get("traffic_bytes_per_row", 0), n.get("traffic_gbs", 0),
                      n.get("traffic_frac", 0), n["frac"], n["frac_basis"].split(" ")[0], " (formula exceeds ceiling)" if n["formula_exceeds_ceiling"] else ""))


if __name__ == "__main__":
    main(sys.argv[1:] or ["main", "c2_s0.01", "c2_s0.99"])

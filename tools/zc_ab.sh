#!/bin/bash
# A/B of zero-copy inputs on the small host-batch calls (host_batch.cpp
# DFMI_HOST_ZC): the batches bench lines, alternating variants twice.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for zc in ${VARIANTS:-0 1}; do
    DFMI_HOST_ZC=$zc timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --sweep "" --extra batches \
        --gather 0 > gpurun_out/zc_$zc.json 2> gpurun_out/zc_$zc.err || { tail -20 gpurun_out/zc_$zc.err; exit 1; }
    python3 - $zc $rep <<'PY' | tee -a gpurun_out/zc_ab.log
import json, sys
zc, rep = sys.argv[1], sys.argv[2]
b = json.load(open("gpurun_out/zc_%s.json" % zc))["extra"]["batches"]
r = b["relation_1024_host"]
print("rep %s ZC=%s  1024_rows_host %.2f us  x256 %.3f us/batch  relation pull %.3f us/batch (%.3g rows/s)  columns %.3f  gate %s" % (
    rep, zc, b["1024_rows_host"]["us_per_batch"], b["1024_rows_host_x256_coalesced"]["us_per_batch"],
    r["pull"]["us_per_batch"], r["pull"]["rows_per_s"], r["pull_and_columns"]["us_per_batch"],
    r["parity_gate"]["bit_identical_to_oracle"] and b["1024_rows_host_x256_coalesced"]["matches_single_batch_calls"]))
PY
  done
done

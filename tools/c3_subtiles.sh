#!/bin/bash
# C3 sub-tile / gather sweep: both C3 queries on one
# 1.25e8-row batch per variant -- DFMI_SUBTILES (sub-tiles per look-back;
# 1 = round 2's one look-back per 2048-row tile), DFMI_OUT_SLICES (slices per
# output step), DFMI_UTF8_GATHER (1 = binary-search emitter, 4 = LDS image,
# 5 = marker scan), DFMI_UTF8_PRESTAGE=1 (first staging round before the
# look-back), the look-back skipped (DFMI_DEBUG_MODE=2: wrong offsets, same
# traffic) and the byte copies skipped (DFMI_DEBUG_MODE=8).
set -o pipefail
mkdir -p gpurun_out
V=${C3_VARIANTS:-"- DFMI_UTF8_GATHER=5 DFMI_UTF8_GATHER=1 DFMI_UTF8_PRESTAGE=1 DFMI_UTF8_GATHER=5,DFMI_UTF8_PRESTAGE=1 DFMI_SUBTILES=1 DFMI_SUBTILES=1,DFMI_OUT_SLICES=2 DFMI_DEBUG_MODE=2 DFMI_DEBUG_MODE=8 -"}
timeout -k 10 400 python -u tools/c3_probe.py $V > gpurun_out/c3_subtiles.log 2>&1
rc=$?; cat gpurun_out/c3_subtiles.log; exit $rc

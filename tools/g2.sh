#!/bin/bash
# Focused GPU check: Utf8 and aggregate parity, then the C3 gather sweep.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k utf8 tests/test_gpu_aggregate.py > gpurun_out/t_g2.log 2>&1
rc=$?; tail -15 gpurun_out/t_g2.log; [ $rc -ne 0 ] && exit $rc
C3_VARIANTS=${C3_VARIANTS:-"- DFMI_UTF8_ARENA=128,DFMI_WAVES_PER_EU=8 DFMI_UTF8_ARENA=192,DFMI_UTF8_IMAGE=65,DFMI_WAVES_PER_EU=8 DFMI_UTF8_ARENA=128 DFMI_UTF8_ARENA=192,DFMI_UTF8_IMAGE=65 DFMI_DEBUG_MODE=8 -"} bash tools/c3_subtiles.sh

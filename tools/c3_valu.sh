#!/bin/bash
# VALU / SALU / LDS instruction counts of the C3 kernels per tools/c3_probe.py
# variant (one rocprofv3 pass; divide by SQ_WAVES for per-wave figures).
# usage: tools/c3_valu.sh <tag> <variant...>
set -o pipefail
TAG=${1:-c3valu}; shift
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
C3_PROBE_WARM=0 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/p1 -o p1 -- python3 $R/tools/c3_probe.py "$@" > $OUT/p1.log 2> $OUT/p1.err || { tail -5 $OUT/p1.err; exit 1; }
find $OUT -name "*.csv"

#!/bin/bash
# SQ / TA counter passes over tools/c3_probe.py variants (one pass per counter group).
# usage: tools/c3_pmc.sh <tag> <variant...>
set -o pipefail
TAG=${1:-c3pmc}; shift
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
for G in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d $OUT/p$i -o p$i -- python3 $R/tools/c3_probe.py "$@" > $OUT/p$i.log 2> $OUT/p$i.err || { tail -5 $OUT/p$i.err; exit 1; }
done
find $OUT -name "*.csv"

#!/bin/bash
# Instruction-cache counters of the C3 kernels (tools/c3_probe.py variants):
# SQC_ICACHE_* / SQ_IFETCH next to the wave cycles, one rocprofv3 pass.
# usage: tools/c3_icache.sh <tag> <variant...>
set -o pipefail
TAG=${1:-c3icache}; shift
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
  --output-format csv -d $OUT/p1 -o p1 -- python3 $R/tools/c3_probe.py "$@" > $OUT/p1.log 2> $OUT/p1.err || { tail -5 $OUT/p1.err; exit 1; }
find $OUT -name "*.csv"

#!/bin/bash
# C3 counters (verdict r01 item 3): probe variants, a rocprofv3 kernel trace
# and FETCH_SIZE / WRITE_SIZE passes of both C3 queries on one 1.25e8-row batch.
# usage: tools/c3_counters.sh <tag> [variants...]
set -o pipefail
TAG=${1:-c3}; shift
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python tools/c3_probe.py "$@" > $OUT/probe.log 2> $OUT/probe.err || { tail $OUT/probe.err; exit 1; }
cat $OUT/probe.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $R/tools/c3_probe.py - > $OUT/kt_probe.log 2> $OUT/kt.err || { tail $OUT/kt.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $R/tools/c3_probe.py - > $OUT/fetch_probe.log 2> $OUT/fetch.err || { tail $OUT/fetch.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 $R/tools/c3_probe.py - > $OUT/write_probe.log 2> $OUT/write.err || { tail $OUT/write.err; exit 1; }
find $OUT -name "*.csv"

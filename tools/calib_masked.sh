#!/bin/bash
# Lane-masked load calibration on one MI355X (tools/membw_masked.hip): the
# timed table, a rocprofv3 kernel trace, and a FETCH_SIZE PMC pass of its own.
# usage: tools/calib_masked.sh <out dir>
set -o pipefail
R=$(pwd)
OUT=$R/${1:-gpurun_out/calib}
mkdir -p $OUT
B=$R/tools/bin/membw_masked
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $B > $OUT/table.txt 2>&1 || { cat $OUT/table.txt; exit 1; }
cat $OUT/table.txt
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- $B > $OUT/kt.log 2>&1 || { tail $OUT/kt.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- $B > $OUT/fetch.log 2>&1 || { tail $OUT/fetch.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $OUT/rdreq -o rdreq -- $B > $OUT/rdreq.log 2>&1 || { tail $OUT/rdreq.log; exit 1; }
find $OUT -name '*.csv' | head -20

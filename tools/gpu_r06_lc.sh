#!/bin/bash
# Round 6: kernel trace of the GROUP BY probe at 4 and 16 Float64 keys (1e8 rows, reused state).
R=$(pwd)
OUT=$R/${1:-gpurun_out/r06_lc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $R/tools/groupby_probe.py 1e8 --no-host --sweep --reuse --card=4,16 > $OUT/probe.log 2> $OUT/kt.err || { tail $OUT/kt.err; exit 1; }
cat $OUT/probe.log | grep -v "^/opt"
grep "gb::" $OUT/kt/*kernel_stats.csv | cut -d, -f1-4

#!/bin/bash
# Round 6: the GROUP BY cardinality sweep on a reused state (table grown once), 1e7 and 1e8 rows.
R=$(pwd)
OUT=$R/${1:-gpurun_out/r06_y}
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/groupby_probe.py 1e7 --no-host --sweep --phases --reuse > $OUT/sweep_1e7.log 2>&1 || { cat $OUT/sweep_1e7.log; exit 1; }
grep -v "^/opt" $OUT/sweep_1e7.log
timeout -k 10 400 python3 -u tools/groupby_probe.py 1e8 --no-host --sweep --phases --reuse --card=4,100,10000,100000,1000000 > $OUT/sweep_1e8.log 2>&1
rc=$?
grep -v "^/opt" $OUT/sweep_1e8.log
exit $rc

#!/bin/bash
# Round 6: GROUP BY phase profile (DFMI_FINISH_PROFILE) at 1e8 rows, 10k keys.
R=$(pwd)
OUT=$R/${1:-gpurun_out/r06_m}
mkdir -p $OUT
DFMI_DIAG=1 DFMI_FINISH_PROFILE=1 timeout -k 10 300 python3 -u tools/groupby_probe.py 1e8 --no-host --sweep --card=10000,1000000 --phases > $OUT/phases.log 2>&1
rc=$?
grep -v "^/opt" $OUT/phases.log | tail -40
exit $rc

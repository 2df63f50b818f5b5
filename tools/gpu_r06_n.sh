#!/bin/bash
# Round 6: GROUP BY suites, then the phase profile at 1e8 rows (10k / 1M keys) and the 1e7 sweep.
R=$(pwd)
OUT=$R/${1:-gpurun_out/r06_n}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_groupby_hash.py tests/test_gpu_aggregate.py tests/test_shard_abi_gpu.py > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
DFMI_DIAG=1 DFMI_FINISH_PROFILE=1 timeout -k 10 300 python3 -u tools/groupby_probe.py 1e8 --no-host --sweep --card=10000,1000000 --phases > $OUT/phases.log 2>&1 || { tail -20 $OUT/phases.log; exit 1; }
grep -v "^/opt" $OUT/phases.log | tail -24
timeout -k 10 300 python3 -u tools/groupby_probe.py 1e7 --no-host --sweep --phases > $OUT/sweep.log 2>&1
rc=$?
grep -v "^/opt" $OUT/sweep.log
exit $rc

#!/bin/bash
# Round 6: GROUP BY suites with the flat finish, then the cardinality sweep and the probe (device only).
R=$(pwd)
OUT=$R/${1:-gpurun_out/r06_f}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_groupby_hash.py tests/test_gpu_aggregate.py tests/test_shard_abi_gpu.py > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python3 -u tools/groupby_probe.py 1e7 --no-host --sweep > $OUT/sweep.log 2>&1 || { cat $OUT/sweep.log; exit 1; }
cat $OUT/sweep.log
timeout -k 10 400 python3 -u tools/groupby_probe.py 1e7 --no-host > $OUT/probe.log 2>&1
rc=$?
cat $OUT/probe.log
exit $rc

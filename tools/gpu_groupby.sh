#!/bin/bash
# Round-6 device GROUP BY check on one MI355X: the hash-table parity tests,
# the aggregate / shard suites that go through it, then the throughput probe.
# Each step under its own time limit; a timeout / crash stops the script.
R=$(pwd)
OUT=$R/${1:-gpurun_out/r06_gb}
mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_groupby_hash.py tests/test_gpu_aggregate.py tests/test_shard_abi_gpu.py > $OUT/pytest.log 2>&1
rc=$?
tail -5 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 400 python3 -u tools/groupby_probe.py > $OUT/probe.log 2>&1
rc2=$?
cat $OUT/probe.log
exit $(( rc > rc2 ? rc : rc2 ))

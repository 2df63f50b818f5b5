#!/bin/bash
# Round 6: GROUP BY suites again (after the NULL-count record change), the
# probe under a rocprofv3 kernel trace, and C3 `!=` variants (tools/c3_probe.py).
R=$(pwd)
OUT=$R/${1:-gpurun_out/r06_b}
mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_groupby_hash.py tests/test_gpu_aggregate.py tests/test_shard_abi_gpu.py > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/gbprof -o gb -- python3 $R/tools/groupby_probe.py 1e7 --no-host > $OUT/probe.log 2>&1 || { tail $OUT/probe.log; exit 1; }
cat $OUT/probe.log
cd $R
C3_PROBE_NE=1 timeout -k 10 400 python3 -u tools/c3_probe.py - DFMI_UTF8_PRESTAGE=1 DFMI_ROWS_PER_THREAD=4 DFMI_UTF8_PRESTAGE=2 > $OUT/c3ne.log 2>&1
rc2=$?
cat $OUT/c3ne.log
exit $(( rc > rc2 ? rc : rc2 ))

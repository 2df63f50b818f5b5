#!/bin/bash
# Round 6: the device finish (k_group_round) -- GROUP BY suites, the probe with
# phases at 1e5 / 1e6 keys, and a kernel trace of the bench's GROUP BY line.
R=$(pwd)
OUT=$R/${1:-gpurun_out/r06_g}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_groupby_hash.py tests/test_gpu_aggregate.py tests/test_shard_abi_gpu.py > $OUT/pytest.log 2>&1
rc=$?
tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 -u tools/groupby_probe.py 1e7 --no-host --sweep --phases > $OUT/sweep.log 2>&1 || { cat $OUT/sweep.log; exit 1; }
cat $OUT/sweep.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o gb -- python3 $R/bench.py --steps 3 --warmup 1 --extra groupby > $OUT/bench_gb.json 2> $OUT/bench_gb.err
rc=$?
tail -c 1500 $OUT/bench_gb.err
exit $rc

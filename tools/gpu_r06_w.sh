#!/bin/bash
# Round 6: claim-limit check variants -- GROUP BY suites (hash file), the 1e7 sweep, the bench GROUP BY line.
R=$(pwd)
OUT=$R/${1:-gpurun_out/r06_w}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_groupby_hash.py > $OUT/pytest.log 2>&1
rc=$?
tail -2 $OUT/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 -u tools/groupby_probe.py 1e7 --no-host --sweep --phases > $OUT/sweep.log 2>&1 || { cat $OUT/sweep.log; exit 1; }
grep -v "^/opt" $OUT/sweep.log
timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 --extra groupby > $OUT/bench_gb.json 2> $OUT/bench_gb.err

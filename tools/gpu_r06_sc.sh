#!/bin/bash
# Round 6: GROUP BY suites + kernel trace of the bench GROUP BY line (scatter A/B).
R=$(pwd)
OUT=$R/${1:-gpurun_out/r06_sc}
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_groupby_hash.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --extra groupby > $OUT/bench.json 2> $OUT/kt.err || { tail $OUT/kt.err; exit 1; }
grep "gb::" $OUT/kt/*kernel_stats.csv | cut -d, -f1-4 | head -8

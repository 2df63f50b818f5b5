#!/bin/bash
# Round 6: the bench's GROUP BY line under a rocprofv3 kernel trace, then C3 `!=` variants.
R=$(pwd)
OUT=$R/${1:-gpurun_out/r06_c}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/gbprof -o gb -- python3 $R/bench.py --steps 3 --warmup 1 --rows 1e8 --sweep 0.5 --no-cpu --gather 0 --extra groupby > $OUT/bench_gb.json 2> $OUT/bench_gb.err || { tail -30 $OUT/bench_gb.err; exit 1; }
cat $OUT/bench_gb.json
cd $R
C3_PROBE_NE=1 timeout -k 10 600 python3 -u tools/c3_probe.py - DFMI_UTF8_EQ_REG=4 DFMI_UTF8_EQ_REG=8 DFMI_UTF8_EQ_REG=2 DFMI_UTF8_PRESTAGE=1 DFMI_ROWS_PER_THREAD=4 - > $OUT/c3ne.log 2>&1
rc=$?
cat $OUT/c3ne.log
exit $rc

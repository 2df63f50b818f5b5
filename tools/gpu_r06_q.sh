#!/bin/bash
# Round 6: long-string gather (tools/long_utf8_probe.py, 1e7 rows of 40-200 B): kernel trace,
# FETCH_SIZE / WRITE_SIZE passes (tools/traffic.py) and one SQ pass, to find its bound.
R=$(pwd)
OUT=$R/${1:-gpurun_out/r06_q}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $R/tools/long_utf8_probe.py > $OUT/kt.log 2> $OUT/kt.err || { tail -5 $OUT/kt.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $R/tools/long_utf8_probe.py > $OUT/fetch.log 2> $OUT/fetch.err || { tail -5 $OUT/fetch.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 $R/tools/long_utf8_probe.py > $OUT/write.log 2> $OUT/write.err || { tail -5 $OUT/write.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU --output-format csv -d $OUT/sq -o sq -- python3 $R/tools/long_utf8_probe.py > $OUT/sq.log 2> $OUT/sq.err || { tail -5 $OUT/sq.err; exit 1; }
cd $R && python3 tools/traffic.py $OUT > $OUT/traffic.txt 2>&1; tail -20 $OUT/traffic.txt
cat $OUT/kt.log

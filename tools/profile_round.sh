#!/bin/bash
# Round profile on one MI355X: GPU parity suite, the default bench line (with
# the CPU baseline), a rocprofv3 kernel-trace of the headline configuration,
# and separate FETCH_SIZE / WRITE_SIZE PMC passes (MI355X_MICROARCH.md
# "rocprofv3 PMC slots": the two do not fit one pass).
# usage: tools/profile_round.sh <tag>
set -o pipefail
TAG=${1:-rNN}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --durations=15 --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $R/bench.py --steps 20 --warmup 3 --sweep 0.5 --no-cpu --extra '' > $OUT/kt_bench.json 2> $OUT/kt.err || { tail $OUT/kt.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $R/bench.py --steps 3 --warmup 1 --sweep 0.5 --no-cpu --extra '' > $OUT/fetch_bench.json 2> $OUT/fetch.err || { tail $OUT/fetch.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 $R/bench.py --steps 3 --warmup 1 --sweep 0.5 --no-cpu --extra '' > $OUT/write_bench.json 2> $OUT/write.err || { tail $OUT/write.err; exit 1; }
find $OUT -name "*.csv" | head -20

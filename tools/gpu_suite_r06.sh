#!/bin/bash
# Round 6: the whole -m gpu suite, then smoke() (one gpurun call).
R=$(pwd)
OUT=$R/${1:-gpurun_out/r06_suite}
mkdir -p $OUT
timeout -k 10 1050 python3 -u -m pytest tests -m gpu -x -v --durations=30 --timeout 300 --timeout-method thread > $OUT/pytest_gpu_all.log 2>&1
rc=$?
tail -5 $OUT/pytest_gpu_all.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log

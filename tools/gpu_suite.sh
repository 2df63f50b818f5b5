#!/bin/bash
# GPU parity suite + smoke + short bench with the query-compiled kernels
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest12.log 2>&1
rc=$?; tail -5 gpurun_out/pytest12.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke12.log 2>&1 || { cat gpurun_out/smoke12.log; exit 1; }
cat gpurun_out/smoke12.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/bench12.json 2> gpurun_out/bench12.err || { tail gpurun_out/bench12.err; exit 1; }
cat gpurun_out/bench12.json

#!/bin/bash
# Host-buffer path check: the GPU parity suite of test_gpu_parity.py (every
# case also through dfmi_filter_project_host, single-chunk and 512-row
# pipelined chunks) and the bench host line (pageable and pinned inputs).
# usage: tools/host_check.sh <tag>
set -o pipefail
TAG=${1:-host}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -15 gpurun_out/$TAG/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --sweep 0.5 --no-cpu --extra host > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail gpurun_out/$TAG/bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/$TAG/bench.json').read().splitlines()[-1]);print(json.dumps(d['extra']))"

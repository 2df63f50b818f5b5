#!/bin/bash
# Full GPU suite, the per-call probe (phase breakdown), then the batches and
# csv bench lines. usage: tools/call_check.sh <tag>
set -o pipefail
TAG=${1:-call}
mkdir -p gpurun_out/$TAG
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/$TAG/pytest.log; [ $rc -ne 0 ] && exit $rc
DFMI_DIAG=1 DFMI_CALL_PROFILE=1 timeout -k 10 120 python tools/call_probe.py > gpurun_out/$TAG/call_probe.log 2>&1 || { tail gpurun_out/$TAG/call_probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/$TAG/call_probe.log | tail -8
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --sweep 0.5 --no-cpu --extra batches,csv > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail gpurun_out/$TAG/bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/$TAG/bench.json').read().splitlines()[-1]);print(json.dumps(d['extra']))"

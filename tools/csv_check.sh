#!/bin/bash
# CSV ingest check: end-to-end CSV / serde / parity GPU tests, then the csv
# and host bench lines. usage: tools/csv_check.sh <tag>
set -o pipefail
TAG=${1:-csv}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests/test_gpu_csv.py tests/test_gpu_serde.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -4 gpurun_out/$TAG/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --sweep 0.5 --no-cpu --extra csv,host > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail gpurun_out/$TAG/bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/$TAG/bench.json').read().splitlines()[-1]);print(json.dumps(d['extra']))"

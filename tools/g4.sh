#!/bin/bash
# Coalesced batches (HBM and host) parity, then the batches bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_batches.py > gpurun_out/t_g4.log 2>&1
rc=$?; tail -4 gpurun_out/t_g4.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --gather 0 --sweep 0.5 --extra batches > gpurun_out/b_g4.json 2> gpurun_out/b_g4.err || { tail gpurun_out/b_g4.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/b_g4.json').read().strip().splitlines()[-1]); print(json.dumps(d['extra']['batches'], indent=1))"

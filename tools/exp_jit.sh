#!/bin/bash
# Tile-shape / look-back experiments on the query-compiled C2 kernel.
# usage: tools/exp_jit.sh [--parity] name:ENV=V,ENV=V ...
set -o pipefail
mkdir -p gpurun_out
if [ "$1" = "--parity" ]; then
  shift
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/exp_pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/exp_pytest.log; [ $rc -ne 0 ] && exit $rc
fi
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  env ${envs//,/ } timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu --extra '' > gpurun_out/exp_$name.json 2> gpurun_out/exp_$name.err || { tail -3 gpurun_out/exp_$name.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/exp_$name.json')); print('$name', ' '.join('%s:%.3f'%(k,v['kernel_ms']) for k,v in d['sweep'].items()))"
done

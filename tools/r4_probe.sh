#!/bin/bash
# Round-4 probe (one gpurun call): the batches / relation parity tests, the
# Utf8 parity cases (C3 gather launch shape), then the per-call bench lines.
# usage: tools/r4_probe.sh [tag] [pytest -k expression]
set -o pipefail
TAG=${1:-probe}
K=${2:-}
mkdir -p gpurun_out
ARGS=(${FILES:-tests/test_gpu_batches.py tests/test_gpu_parity.py})
[ -n "$K" ] && ARGS+=(-k "$K")
timeout -k 10 ${PT_TIMEOUT:-600} python -u -m pytest -x -v --timeout 120 --timeout-method thread "${ARGS[@]}" \
    > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_$TAG.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu --sweep "" --extra ${EXTRA:-batches,c3} --gather 0 \
    > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
python -c "
import json,sys
d=json.load(open('gpurun_out/bench_$TAG.json'))
b=d['extra']['batches']
print('headline', d['ms_per_step'], d['roofline']['frac'])
for k in ('1024_rows','1048576_rows','1024_call_after_full_table_us','1024_rows_host','1024_rows_host_x256_coalesced','1024_rows_x256_coalesced','relation_1024_host'):
    print(k, json.dumps(b.get(k)))
for q in (('eq','lt') if 'c3' in d['extra'] else ()):
    print('c3', q, d['extra']['c3'][q]['kernel_ms'], d['extra']['c3'][q]['roofline']['kernel'])
"

#!/bin/bash
# Utf8 path check: the parity suites over Utf8 / all types, then the C3
# probe over the given variants.
# usage: tools/c3_check.sh <tag> [variants...]
set -o pipefail
TAG=${1:-c3check}; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_types.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/$TAG/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/c3_probe.py "$@" > gpurun_out/$TAG/probe.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/$TAG/probe.log; exit $rc

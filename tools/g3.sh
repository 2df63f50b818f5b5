#!/bin/bash
# Utf8 gather variants' parity, then the same-box C3 A/B against _ab/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "gather_variants or subtile or utf8_gather_and or utf8_many or multi_channel" > gpurun_out/t_g3.log 2>&1
rc=$?; tail -4 gpurun_out/t_g3.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_c3.sh "$@"

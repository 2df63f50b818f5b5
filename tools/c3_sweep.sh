#!/bin/bash
# C3 rows-per-thread sweep (diagnostics): tools/c3_sweep.sh <tag>
set -o pipefail
export DFMI_DIAG=1  # the library reads its diagnostic knobs only then
mkdir -p gpurun_out
for K in 8 4 2; do
  DFMI_ROWS_PER_THREAD=$K timeout -k 10 200 python bench.py --rows 1e7 --steps 5 --warmup 1 --sweep 0.5 --no-cpu --extra c3 > gpurun_out/c3_$1_k$K.json 2> gpurun_out/c3_$1_k$K.err || exit 1
  python -c "import json,sys; c=json.load(open(sys.argv[1]))['extra']['c3']; print(sys.argv[1], c['eq']['kernel_ms'], c['lt']['kernel_ms'])" gpurun_out/c3_$1_k$K.json
done

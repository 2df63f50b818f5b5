#!/bin/bash
# Tile-shape sweep (diagnostics): C2 s=0.5 + C3 at (BLOCK, K) pairs.
set -o pipefail
export DFMI_DIAG=1  # the library reads its diagnostic knobs only then
mkdir -p gpurun_out
for BK in 512:8 256:8 256:16; do
  B=${BK%:*}; K=${BK#*:}
  DFMI_BLOCK=$B DFMI_ROWS_PER_THREAD=$K timeout -k 10 240 python bench.py --steps 10 --warmup 2 --sweep 0.5 --no-cpu --extra c3 > gpurun_out/shape_${B}_$K.json 2> gpurun_out/shape_${B}_$K.err || { tail -3 gpurun_out/shape_${B}_$K.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['extra']['c3']; print(sys.argv[1], d['roofline']['kernel_ms'], 'c3', c['eq']['kernel_ms'], c['lt']['kernel_ms'])" gpurun_out/shape_${B}_$K.json
done

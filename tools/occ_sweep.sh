#!/bin/bash
# Occupancy-hint sweep (diagnostics): C2 sweep + C3 at DFMI_WAVES_PER_EU=0/8.
set -o pipefail
export DFMI_DIAG=1  # the library reads its diagnostic knobs only then
mkdir -p gpurun_out
for W in 0 8; do
  DFMI_WAVES_PER_EU=$W timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu --extra c3,c4 > gpurun_out/occ_w$W.json 2> gpurun_out/occ_w$W.err || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['extra']['c3']; print(sys.argv[1], {k:v['kernel_ms'] for k,v in d['sweep'].items()}, 'c4', d['extra']['c4']['kernel_ms'], 'c3', c['eq']['kernel_ms'], c['lt']['kernel_ms'])" gpurun_out/occ_w$W.json
done

#!/bin/bash
# A/B of the aggregate kernel's sub-tile form on the Q6 line: M forced by the
# diagnostic knob (1 = one tile per block) and d = the adaptive default.
set -o pipefail
for rep in 1 2; do for v in 1 2 4 d; do
  if [ $v = d ]; then E=""; else E="DFMI_DIAG=1 DFMI_AGG_SUBTILES=$v"; fi
  env $E timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --sweep "" --no-cpu --extra q6 --gather 0 > gpurun_out/q6_$v.json 2> gpurun_out/q6_$v.err || { tail gpurun_out/q6_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/q6_$v.json'))['extra']['q6']
print('rep $rep M=$v', d.get('kernel_ms'), d['roofline']['kernel'], d.get('parity_gate'))" | tee -a gpurun_out/q6_ab.log
done; done

#!/bin/bash
# A/B of the numeric sub-tile kernel (exec.cpp kLowSel / jit.cpp "M
# sub-tiles") on the low-selectivity lines: C2 at s = 1% and C4, forced per
# variant with the diagnostic knob (DFMI_DIAG=1 DFMI_NUMERIC_SUBTILES=M; M=1:
# the one-tile kernel, the adaptive choice disabled with DFMI_NUMERIC_SUBTILES=1),
# alternating variants twice on the same box; variant d = the adaptive default.
# usage: tools/ab_subtiles.sh [out file] [variants...]
set -o pipefail
OUT=${1:-gpurun_out/ab_subtiles.log}
shift
VARIANTS=${@:-1 8 4 2}
mkdir -p $(dirname $OUT)
: > $OUT
for rep in 1 2; do
  for m in $VARIANTS; do
    if [ "$m" = d ]; then E=""; else E="DFMI_DIAG=1 DFMI_NUMERIC_SUBTILES=$m"; fi  # d: the adaptive default
    env $E timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --sel 0.01 \
        --sweep 0.01 --no-cpu --extra c4 --gather 0 > gpurun_out/ab_sub_$m.json 2> gpurun_out/ab_sub_$m.err \
        || { tail gpurun_out/ab_sub_$m.err; exit 1; }
    python3 - $m $rep >> $OUT <<'EOF'
import json, sys
m, rep = sys.argv[1], sys.argv[2]
d = json.load(open("gpurun_out/ab_sub_%s.json" % m))
c4 = d["extra"]["c4"]
print("rep %s M=%s  C2 s=1%%: kernel %.4f ms (%s)  C4: kernel %.4f ms (%s)  gates %s %s" % (
    rep, m, d["roofline"]["kernel_ms"], d["roofline"]["kernel"], c4["kernel_ms"], c4["roofline"]["kernel"],
    d["parity_gate"]["bit_identical_to_oracle"], c4["parity_gate"]["bit_identical_to_oracle"]))
EOF
    tail -1 $OUT
  done
done

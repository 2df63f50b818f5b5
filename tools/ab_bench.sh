#!/bin/bash
# Same-box A/B of the C2 / C3 bench lines: the previous commit's tree (_ab/,
# a git worktree built in the container; not committed) against this tree,
# alternating, so box-to-box spread does not enter the
# comparison.
set -o pipefail
mkdir -p gpurun_out
for it in 1 2; do
  for side in _ab .; do
    timeout -k 10 200 python -u $side/bench.py --steps 20 --warmup 3 --no-cpu --gather 0 --extra "${AB_EXTRA:-}" --sweep 0.5 \
      > gpurun_out/ab_${side//[._\/]/}_$it.json 2> gpurun_out/ab_err.log || { tail gpurun_out/ab_err.log; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_ms'])" gpurun_out/ab_${side//[._\/]/}_$it.json "$side#$it"
  done
done

#!/bin/bash
# Same-box A/B of the two C3 queries: the tree in _ab/ (a git worktree of an
# earlier commit, built in the container; not committed) against this tree,
# alternating; extra args are c3_probe variants for this tree.
set -o pipefail
mkdir -p gpurun_out
for it in 1 2; do
  (cd _ab && timeout -k 10 200 python -u tools/c3_probe.py -) 2>&1 | grep -v amdgpu.ids | sed "s/^/_ab#$it /" || exit 1
  timeout -k 10 300 python -u tools/c3_probe.py - "$@" 2>&1 | grep -v amdgpu.ids | sed "s/^/.#$it /" || exit 1
done

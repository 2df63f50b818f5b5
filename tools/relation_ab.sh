#!/bin/bash
# bench.py's relation_1024_host line alone, once per DFMI_HOST_THREADS value
# (each its own process: the packing pool is sized at first use).
# usage: tools/relation_ab.sh <threads...>
for t in "$@"; do
  DFMI_HOST_THREADS=$t timeout -k 10 120 python3 -c "
import json, sys
sys.path.insert(0, 'tests')
import bench
r = bench.relation_host_line(0.5)
print('threads $t', 'pull_and_columns %.3f us' % r['pull_and_columns']['us_per_batch'], 'pull %.3f us' % r['pull']['us_per_batch'],
      'rust %.3f us' % r['rust_binding_path']['us_per_batch'])
" || exit 1
done

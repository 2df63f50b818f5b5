#!/bin/bash
# bench.py's relation_1024_host line alone at several read-ahead group sizes
# (coalesce = batches per native call), alternating, one process.
# usage: tools/relation_coalesce_ab.sh <coalesce...>
timeout -k 10 400 python3 -c "
import sys
sys.path.insert(0, 'tests')
import bench
for co in [int(x) for x in sys.argv[1:]]:
    r = bench.relation_host_line(0.5, coalesce=co)
    print('coalesce %4d' % co, 'pull_and_columns %.3f us' % r['pull_and_columns']['us_per_batch'],
          'pull %.3f us' % r['pull']['us_per_batch'], flush=True)
" "$@"

#!/bin/bash
# bench.py's relation_1024_host line alone under environment variants, one
# process each (the library reads some knobs once per process).
# usage: tools/relation_env_ab.sh "-" "DFMI_HOST_ZC=0" ...   ('-' = none)
for v in "$@"; do
  if [ "$v" = "-" ]; then envs=""; else envs="$v"; fi
  env $envs timeout -k 10 150 python3 -c "
import sys
sys.path.insert(0, 'tests')
import bench
r = bench.relation_host_line(0.5)
print('%-28s' % '$v', 'pull_and_columns %.3f us' % r['pull_and_columns']['us_per_batch'], 'pull %.3f us' % r['pull']['us_per_batch'],
      'rust %.3f us' % r['rust_binding_path']['us_per_batch'], flush=True)
" || exit 1
done

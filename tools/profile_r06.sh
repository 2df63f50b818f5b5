#!/bin/bash
# Round-6 profile of every bench line on one MI355X: for each
# run -- main (C2 s=0.5 + C4 + Q6 + C2 Int64 + C3 + batches), c2_s0.01 (+ C4: the
# low-selectivity sub-tile kernels), c2_s0.99 -- a
# rocprofv3 kernel trace of the bench command, then separate FETCH_SIZE and
# WRITE_SIZE PMC passes of the same command (MI355X_MICROARCH.md: the two do
# not fit one pass), reduced by tools/traffic.py to <run>/traffic.json, which
# bench.py reads (roofline.rocprof / roofline.traffic of every line).
# usage: tools/profile_r06.sh <out dir, e.g. gpurun_out/r06> [runs...]
set -o pipefail
R=$(pwd)
OUT=$R/${1:-gpurun_out/r06}
shift
RUNS=${@:-main c2_s0.01 c2_s0.99}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for run in $RUNS; do
  case $run in
    main) ARGS="--steps 10 --warmup 2 --sweep 0.5 --no-cpu --extra c4,q6,c2i64,c3,groupby,batches";;
    c2_s0.01) ARGS="--steps 10 --warmup 2 --sel 0.01 --sweep 0.01 --no-cpu --extra c4";;
    c2_s*) S=${run#c2_s}; ARGS="--steps 10 --warmup 2 --sel $S --sweep $S --no-cpu --extra ''";;
    *) echo "unknown run $run"; exit 2;;
  esac
  D=$OUT/$run
  mkdir -p $D
  # which box: the bench lines carry the same id (bench.py "box"), so a line's HIP-event
  # time and the committed profile it cites can be told apart when they come from two boxes
  timeout -k 10 120 python3 -c "import socket, torch; p = torch.cuda.get_device_properties(0); print(socket.gethostname(), p.name, getattr(p, 'gcnArchName', ''), 'uuid', getattr(p, 'uuid', '?'), 'pci', getattr(p, 'pci_bus_id', '?'))" > $D/box.txt || exit 1
  echo "== $run: $ARGS"
  eval timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o kt -- python3 $R/bench.py $ARGS > $D/bench.json 2> $D/kt.err || { tail $D/kt.err; exit 1; }
  eval timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o fetch -- python3 $R/bench.py $ARGS > $D/fetch_bench.json 2> $D/fetch.err || { tail $D/fetch.err; exit 1; }
  eval timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o write -- python3 $R/bench.py $ARGS > $D/write_bench.json 2> $D/write.err || { tail $D/write.err; exit 1; }
  python3 $R/tools/traffic.py $D || exit 1
done

#!/bin/bash
# Round 6 final checks: the default bench (N=1, cpu_baseline included), then the
# --gpus 2 path rehearsed with two gloo ranks sharing the one GPU (GROUP BY in the extras).
R=$(pwd)
OUT=$R/${1:-gpurun_out/r06_e}
mkdir -p $OUT
timeout -k 10 700 python3 -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
rc=$?
tail -c 2000 $OUT/bench_default.err
if [ $rc -ne 0 ]; then exit $rc; fi
DFMI_BENCH_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 \
  > $OUT/bench_gloo2.json 2> $OUT/bench_gloo2.err
rc=$?
tail -c 2000 $OUT/bench_gloo2.err
exit $rc

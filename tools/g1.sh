set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_shard_abi_gpu.py tests/test_jit_cpu.py > gpurun_out/t1.log 2>&1 || { tail -40 gpurun_out/t1.log; exit 1; }
tail -3 gpurun_out/t1.log
timeout -k 10 500 python -u bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err || { tail -30 gpurun_out/bench1.err; exit 1; }
cat gpurun_out/bench1.json

#!/bin/bash
# GPU-box step runner: gpu_steps.sh "name|seconds|command" ...
# Each step runs under its own time limit with output in gpurun_out/<name>.log.
# A step that times out, aborts or crashes ends the script; for steps named
# pytest* exit status 1 (failed tests) does not -- the next step still runs.
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; secs=${rest%%|*}; cmd=${rest#*|}
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then
    case $name in pytest*) [ $rc -eq 1 ] && continue;; esac
    echo "stopping after $name (rc=$rc)"; exit $rc
  fi
done

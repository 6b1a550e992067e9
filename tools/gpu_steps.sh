#!/bin/bash
# Run GPU steps in order; each under its own time limit. Continue past ordinary test failures
# (pytest rc 1) but stop at anything that suggests a fault, abort, crash or timeout.
# usage: tools/gpu_steps.sh "<seconds>|<name>|<command>" ...
mkdir -p gpurun_out
for step in "$@"; do
  secs="${step%%|*}"; rest="${step#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc"
  tail -n 8 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then
    echo "=== stopping after [$name] (rc=$rc)"; exit $rc
  fi
done

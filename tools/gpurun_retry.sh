#!/bin/bash
# Submit one gpurun call; resubmit ONLY when gpurun reports no box/slot (exit 3, nothing ran).
# usage: tools/gpurun_retry.sh <logfile> <timeout> <command>
log="$1"; to="$2"; shift 2
for attempt in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -ne 3 ]; then echo "gpurun rc=$rc (attempt $attempt)" >> "$log"; exit $rc; fi
  sleep 45
done
echo "gpurun: gave up after repeated exit 3" >> "$log"

#!/bin/bash
# Submit one gpurun call; resubmit ONLY when gpurun reports no box/slot (exit 3, nothing ran),
# waiting out any back-off the client announces ("retry in Ns").
# usage: tools/gpurun_retry.sh <logfile> <timeout> <command>
log="$1"; to="$2"; shift 2
for attempt in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -ne 3 ]; then echo "gpurun rc=$rc (attempt $attempt)" >> "$log"; exit $rc; fi
  wait_s=$(grep -o 'retry in [0-9]*s' "$log" | tail -1 | grep -o '[0-9]*')
  sleep $(( ${wait_s:-60} + 20 ))
done
echo "gpurun: gave up after repeated exit 3" >> "$log"

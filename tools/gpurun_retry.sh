#!/bin/bash
# Submit one gpurun call; resubmit ONLY when gpurun reports that nothing ran (exit 3: no box/slot,
# or status=transient: the box failed while being prepared), waiting out any back-off the client
# announces ("retry in Ns"). A GPU step that ran and failed is never resubmitted.
# usage: tools/gpurun_retry.sh <logfile> <timeout> <command>
log="$1"; to="$2"; shift 2
for attempt in $(seq 1 ${GPURUN_ATTEMPTS:-30}); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q 'status=transient rc=None' "$log"; then
    echo "gpurun rc=$rc (attempt $attempt)" >> "$log"; exit $rc
  fi
  wait_s=$(grep -o 'retry in [0-9]*s' "$log" | tail -1 | grep -o '[0-9]*')
  cp "$log" "$log.attempt$attempt"
  sleep $(( ${wait_s:-60} + 20 ))
done
echo "gpurun: gave up after repeated no-box / transient refusals" >> "$log"

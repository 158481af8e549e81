#!/bin/bash
# Local helper (runs in the build container, not on the GPU box): submit one gpurun call, and
# resubmit it only while gpurun reports that no box/slot is free (nothing ran, nothing charged).
# Usage: scripts/gpurun_when_free.sh LOG TIMEOUT 'command'
log=$1; to=$2; cmd=$3
for attempt in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$log"; then sleep 150; continue; fi
  exit $rc
done
exit 3

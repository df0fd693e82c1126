#!/bin/bash
# Client-side: re-submit a gpurun call only when nothing ran (no box free: exit 3, or a transient
# infrastructure status before the command started). Any other outcome is returned as is.
# usage: tools/gpurun_retry.sh <timeout> '<command>' <log>
to=$1; cmd=$2; log=$3
for i in $(seq 1 ${GPURUN_TRIES:-8}); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient rc=None" "$log"; then
    echo "attempt $i: no box ($rc), retrying in 150 s" >> "$log.retries"
    sleep ${GPURUN_SLEEP:-150}
    continue
  fi
  exit $rc
done
exit 3

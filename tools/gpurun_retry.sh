#!/bin/bash
# gpurun with retries on infrastructure-side transients only (no box or slot
# free, box lost while being prepared): the command itself never ran, so
# nothing is re-run after a failure of the command.  Usage:
#   tools/gpurun_retry.sh LOG TIMEOUT 'command'
log=$1; to=$2; shift 2
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient" "$log" && grep -q "run 0.0s\|run Nones" "$log"; then
    sleep 60
    continue
  fi
  exit $rc
done
exit $rc

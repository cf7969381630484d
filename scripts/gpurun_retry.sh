#!/bin/bash
# Submit one gpurun call, resubmitting ONLY when nothing ran on a GPU: no slot or
# box free (exit 3), the client's infrastructure back-off, or a transient lease
# failure reported before the command started.  A command that ran and failed is
# never resubmitted.  usage: scripts/gpurun_retry.sh <log> <timeout> <command>
log=$1; to=$2; shift 2
for attempt in $(seq 1 ${ATTEMPTS:-8}); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "backing off\|status=transient" "$log"; then
    w=$(grep -o "retry in [0-9]*s" "$log" | grep -o "[0-9]*" | tail -1)
    sleep $(( ${w:-150} + 20 ))
    continue
  fi
  exit $rc
done
exit $rc

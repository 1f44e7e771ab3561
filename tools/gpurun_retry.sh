#!/bin/bash
# Acquire-retry wrapper around gpurun: re-submits only when the box could not be prepared
# (status=transient / exit 3: nothing ran, nothing charged).  Never retries a command that ran.
# usage: tools/gpurun_retry.sh LOG TIMEOUT 'command'
log=$1; to=$2; shift 2
for attempt in 1 2 3 4 5 6; do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient\|no box\|backing off" "$log" && ! grep -q "status=ok" "$log"; then
    echo "attempt $attempt: transient, retrying in 120 s" >> "$log.retries"
    sleep 120
    continue
  fi
  exit $rc
done
exit 3

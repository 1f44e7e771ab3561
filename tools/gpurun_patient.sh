#!/bin/bash
# Patient acquire-retry wrapper around gpurun: re-submits only while gpurun reports a transient
# (no box / backing off / box lost before the command ran: nothing ran, nothing charged),
# sleeping as long as gpurun asks (default 180 s).  Never retries a command that ran.
# usage: tools/gpurun_patient.sh LOG TIMEOUT MAX_ATTEMPTS 'command'
log=$1; to=$2; max=$3; shift 3
for attempt in $(seq 1 "$max"); do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient" "$log" && ! grep -q "status=ok" "$log"; then
    wait_s=$(grep -o "retry in [0-9]*s" "$log" | tail -1 | grep -o "[0-9]*")
    wait_s=${wait_s:-180}
    echo "attempt $attempt: transient, retrying in $((wait_s + 15)) s" >> "$log.retries"
    sleep $((wait_s + 15))
    continue
  fi
  exit $rc
done
exit 3

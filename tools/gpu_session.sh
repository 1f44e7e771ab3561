#!/bin/bash
# GPU-box session driver: runs steps in order, each under its own time limit.
# Stops at the first fault-class exit (timeout 124/137, abort 134, segv 139, kill 143);
# an ordinary failure (exit 1, e.g. a failed assertion) is recorded and the session goes on.
# usage: tools/gpu_session.sh "<name>|<seconds>|<command>" ...
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] $(date +%T) timeout=${secs}s: $cmd" | tee -a gpurun_out/session.log
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc $(date +%T)" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.log"
  case $rc in
    0|1|2|5) ;;
    *) echo "=== stopping: fault-class exit $rc" | tee -a gpurun_out/session.log; exit $rc ;;
  esac
done

#!/bin/bash
# gpurun with retries while no box/slot is free (exit 3: nothing ran, nothing charged)
# usage: gpr.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  echo "EXIT $rc (try $i)" >> "$LOG"
  [ $rc -ne 3 ] && exit $rc
  sleep 90
done

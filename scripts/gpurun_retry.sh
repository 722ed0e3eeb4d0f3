#!/bin/bash
# Retry a gpurun call while the pool reports a transient/no-box condition (exit 3 or status=transient).
# usage: scripts/gpurun_retry.sh LOGFILE TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient\|no box\|slot free" $LOG || [ $rc -eq 3 ]; then sleep 60; continue; fi
  echo "exit=$rc" >> $LOG; exit $rc
done
echo "exit=giveup" >> $LOG

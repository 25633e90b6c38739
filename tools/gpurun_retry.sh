#!/bin/bash
# Resubmit a gpurun call ONLY while the pool reports an infrastructure event before the command ran
# (box not prepared / taken away / back-off: nothing executed, nothing charged). Any run that
# executed -- pass or fail -- is returned as is. Usage: tools/gpurun_retry.sh <log> <timeout_s> '<cmd>'
log=$1; to=$2; cmd=$3
for i in 1 2 3 4 5 6; do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient\|backing off\|stopped responding while being prepared\|taken away by the GPU service" "$log" && \
     ! grep -q "status=ok" "$log"; then
    sleep 60; continue
  fi
  [ $rc -eq 3 ] && { sleep 90; continue; }
  break
done
tail -3 "$log"

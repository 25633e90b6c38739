#!/bin/bash
# Resubmit a gpurun call ONLY while the pool reports that nothing executed (box not prepared / taken
# away / no box or slot free / back-off: nothing ran, nothing charged). Any run that executed -- pass
# or fail, whatever its exit code -- is returned as is, so a GPU failure is read, not re-run.
# Usage: tools/gpurun_retry.sh <log> <timeout_s> '<cmd>'
log=$1; to=$2; cmd=$3
for i in 1 2 3 4 5 6 7 8 9 10 11 12; do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient\|backing off\|stopped responding while being prepared\|taken away by the GPU service\|no box\|no slot" "$log" && \
     ! grep -q "status=ok\|status=fail" "$log"; then
    if grep -q "backing off" "$log"; then sleep 170; else sleep 90; fi; continue
  fi
  break
done
tail -3 "$log"
exit $rc

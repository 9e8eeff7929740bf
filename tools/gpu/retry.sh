#!/bin/bash
# usage: tools/gpu/retry.sh LOG TIMEOUT script.sh -- re-submits only while gpurun reports that nothing ran
# (no box / slot free, or the box was withdrawn by the service before the command started)
LOG=$1; TO=$2; shift 2
for i in $(seq 1 20); do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout $TO -- bash "$@" > $LOG 2>&1
  if grep -q "no free box right now\|GPU slot(s) on this pod are busy\|backing off\|stopped responding while being prepared\|was taken away by the GPU service" $LOG && ! grep -q "status=ok" $LOG; then
    sleep 120; continue
  fi
  break
done
echo DONE >> $LOG

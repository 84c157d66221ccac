#!/bin/bash
# Run one gpurun call, waiting out "no free box / slots busy / backing off" (nothing
# charged, nothing ran); any other outcome (including a failing command) ends the loop.
#   scripts/gpurun_wait.sh <timeout> <script> [log]
T=$1; S=$2; LOG=${3:-gpurun_out/wait_$(basename $S .sh).log}
mkdir -p gpurun_out
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout $T -- bash $S > $LOG 2>&1
  if grep -q "status=transient" $LOG && grep -qE "no free box|slot\(s\) on this pod are busy|backing off|stopped responding while being prepared" $LOG; then
    sleep 60; continue
  fi
  break
done
echo "done after $i tries" >> $LOG

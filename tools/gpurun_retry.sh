#!/bin/bash
# Retry a gpurun call while the pool has no free box (gpurun exit code 3: nothing ran, nothing
# charged).  Any other exit code ends the loop.  Usage: tools/gpurun_retry.sh OUT TIMEOUT 'cmd'
out=$1; lim=$2; cmd=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$out" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q -e "no free box right now" -e "slot(s) on this pod are busy" -e "status=transient" "$out"; then break; fi
  sleep 120
done
echo "gpurun rc=$rc after $i tries" >> "$out"

#!/usr/bin/env bash
# gpurun with retries ONLY while the pool has no free box (exit 3: nothing ran, nothing charged).
# usage: bash tools/gpurun_retry.sh <log> <timeout_s> '<command>'
log=$1; tmo=$2; cmd=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$tmo" -- "$cmd" > "$log" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "no free box right now\|taken away by the GPU service" "$log"; then exit $rc; fi
  echo "[retry $i: no box, rc=$rc]" >> "$log.retries"
  sleep 150
done
exit $rc

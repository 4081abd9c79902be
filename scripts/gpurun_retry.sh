#!/bin/bash
# Submit one gpurun call; when the pool has no free slot (nothing charged), wait and submit again.
# Usage: scripts/gpurun_retry.sh <timeout> '<command>'
to=$1; shift
for i in $(seq 1 20); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$to" -- "$@" 2>&1)
  echo "$out" | tail -40
  if echo "$out" | grep -q "nothing was charged\|no free box right now\|backing off\|stopped responding while being prepared"; then sleep 150; continue; fi
  exit 0
done

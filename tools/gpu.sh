#!/bin/bash
# gpurun wrapper for this repo's interactive work: re-submits ONLY when gpurun reports that no
# box was prepared (status=transient / exit 3: nothing ran, nothing charged).  A command that
# ran and failed is never re-submitted.   tools/gpu.sh <log> <timeout_s> '<command>'
log=$1; to=$2; shift 2
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  if grep -q "status=transient" "$log" || [ $rc -eq 3 ]; then sleep 20; continue; fi
  exit $rc
done
exit $rc

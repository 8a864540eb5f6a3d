#!/bin/bash
# Re-submit a gpurun call ONLY when gpurun reports that the box never ran it (status=transient / backing off /
# no box free).  A call that ran is never repeated, whatever its outcome.
# usage: tools/gpurun_retry.sh <outfile> <timeout> '<command>'
out=$1; to=$2; cmd=$3
for attempt in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
  rc=$?
  if grep -q "status=transient\|backing off\|no box\|slot free" "$out" && ! grep -q "status=ok" "$out"; then
    echo "[retry] attempt $attempt: box not available (rc=$rc); waiting" >&2
    sleep 60
    continue
  fi
  break
done
tail -6 "$out"

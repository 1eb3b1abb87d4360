#!/bin/bash
# Submit one gpurun command, re-submitting ONLY while the pool reports that nothing ran (no box
# free / infrastructure back-off / box lost while being prepared).  A command that ran -- whatever
# its exit status -- is never re-submitted.
#   tools/gpurun_when_free.sh LOG TIMEOUT 'command'
log=$1; to=$2; cmd=$3
for attempt in 1 2 3 4 5 6 7 8 9 10 11 12; do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  if grep -qE "no free box right now|backing off after the last attempt|stopped responding while being prepared" "$log" \
     && ! grep -qE "status=(ok|fail|timeout|error)" "$log"; then
    echo "[attempt $attempt] nothing ran; waiting" >> "$log.attempts"
    sleep 150
    continue
  fi
  echo "[attempt $attempt] rc=$rc" >> "$log.attempts"
  exit $rc
done
exit 3

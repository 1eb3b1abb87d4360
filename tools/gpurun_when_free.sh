#!/bin/bash
# Submit one gpurun command, re-submitting ONLY while the pool reports that nothing ran (no box
# free / infrastructure back-off / box lost while being prepared).  A command that ran -- whatever
# its exit status -- is never re-submitted.
#   tools/gpurun_when_free.sh LOG TIMEOUT 'command'
# (run a copy -- bash reads a script while it runs: `cp tools/gpurun_when_free.sh /tmp/gw.sh`, with
#  REPO=/root/repo -- so editing the tree's copy never changes a wrapper in flight)
log=$1; to=$2; cmd=$3
REPO=${REPO:-$(cd "$(dirname "$0")/.." && pwd)}
fresh() {  # the in-tree .so was linked from the csrc/ now in the tree (else the GPU run would refuse it)
  (cd "$REPO" && timeout 120 python -c "
from apmbackend_amd import _native
from apmbackend_amd.build_native import csrc_hash
import sys
sys.exit(0 if _native.load(build_if_missing=False).csrc_hash() == csrc_hash() else 1)" 2>/dev/null)
}
for attempt in $(seq 1 ${ATTEMPTS:-40}); do
  while ! fresh; do echo "[attempt $attempt] .so stale (rebuild pending): waiting" >> "$log.attempts"; sleep 30; done
  (cd "$REPO" && /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd") > "$log" 2>&1
  rc=$?
  if grep -qE "no free box right now|backing off after the last attempt|stopped responding while being prepared|nothing was charged" "$log" \
     && ! grep -qE "status=(ok|fail|timeout|error)" "$log"; then
    echo "[attempt $attempt] nothing ran; waiting" >> "$log.attempts"
    sleep 150
    continue
  fi
  echo "[attempt $attempt] rc=$rc" >> "$log.attempts"
  exit $rc
done
exit 3

#!/bin/bash
# Host-join replay throughput at 1 / 8 / 16 concurrent workers (one JVM's synthetic batches
# each), from ordinary and from hipHostMalloc'd (pinned) buffers, to see how the join scales
# with the cores a node gives one GPU process.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=${JOIN_DIR:-/tmp/joinscale}
B=${BATCHES:-24}
mkdir -p gpurun_out
python tools/join_prof.py --batches $B --dir "$D" --hip 2>&1 | tail -1
for pinned in 0 1; do
  for n in ${CONC:-1 8 16}; do
    echo "pinned=$pinned concurrent=$n"
    for i in $(seq $n); do
      (if [ $pinned = 1 ]; then export JOIN_REPLAY_PINNED=1; fi; JOIN_REPLAY_QUIET=1 "$D/join_replay" "$D" $B 2>&1 | tail -1) &
    done
    wait
  done
done
nproc; lscpu | grep -i "model name\|^L[23]\|MHz\|NUMA" || true

#!/bin/bash
# Steady-state headline (200 steps) + kernel stats of the final tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pf; mkdir -p $O
:
:
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1 || exit $?
find $O/prof -name '*kernel_stats.csv' | head -1

#!/bin/bash
# Two default headline benches + smoke on the current tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/b2; mkdir -p $O
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python bench.py > $O/bench_$i.log 2>&1 || exit $?
  tail -1 $O/bench_$i.log | cut -c1-200
done

#!/bin/bash
# Round evidence on the final tree: GPU suite, smoke, driver-shaped bench (20/5) x2, 200-step
# headline, kernel stats.  Each GPU step time-limited; stop at the first crash.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
ok() { case $1 in 0|1) ;; *) echo "stop rc=$1"; exit $1 ;; esac; }
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $O/gpu_suite.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -2 $O/gpu_suite.log; ok $rc
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 $O/smoke.log; ok $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_20_$i.log 2>&1; rc=$?; ok $rc
  tail -1 $O/bench_20_$i.log | cut -c1-140
done
timeout -k 10 300 python bench.py --steps 200 --warmup 5 > $O/headline_200.log 2>&1; rc=$?; ok $rc
tail -1 $O/headline_200.log | cut -c1-140
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1; rc=$?; ok $rc
echo "prof rc=$rc"

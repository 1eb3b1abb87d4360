#!/bin/bash
# GPU suite, headline x2 + kernel stats, then the service path (files -> tailer -> engine -> DB
# sink spool) with 1 / 4 / 8 sink writer lanes.  Every GPU step time-limited; stop at a failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/lanes
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do  # repeat of the K14 70-JVM rollup test (one failure seen on an earlier tree)
  timeout -k 10 120 python -u -m pytest tests/test_engine_gpu.py -q -k "rollup" --timeout 100 --timeout-method thread > $O/rollup_$r.log 2>&1
  rc=$?; tail -1 $O/rollup_$r.log; [ $rc -le 1 ] || exit $rc
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/headline_$i.log 2>&1 || exit $?
  tail -1 $O/headline_$i.log | cut -c1-160
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 3 > $O/prof.log 2>&1 || exit $?
n=0
for l in 1 4 8 1 4 8; do
  n=$((n+1))
  timeout -k 10 300 python bench.py --path service --steps 30 --warmup 3 --writer-lanes $l > $O/service_${n}_l$l.log 2>&1 || exit $?
  tail -1 $O/service_${n}_l$l.log | cut -c1-120
done
echo done

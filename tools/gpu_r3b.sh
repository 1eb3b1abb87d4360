#!/bin/bash
# After K5-on-device: K2 tile kernel re-check (host join), headline line/tile A/B, audit-heavy
# shards, service path, kernel stats.  Each GPU step time-limited; stop at the first crash.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3b; mkdir -p $O
ok() { case $1 in 0|1) ;; *) echo "stop rc=$1"; exit $1 ;; esac; }
APM_PARSE=tile timeout -k 10 200 python -u tools/diag/k5_dump.py edge > $O/tile_edge.log 2>&1; rc=$?
echo "tile edge rc=$rc"; grep seed $O/tile_edge.log; ok $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 60 --warmup 5 > $O/headline_line_$i.log 2>&1; rc=$?; ok $rc
  tail -1 $O/headline_line_$i.log | cut -c1-200
  APM_PARSE=tile timeout -k 10 300 python bench.py --steps 60 --warmup 5 > $O/headline_tile_$i.log 2>&1; rc=$?; ok $rc
  tail -1 $O/headline_tile_$i.log | cut -c1-200
done
for af in 0.10 0.25; do
  timeout -k 10 300 python bench.py --steps 60 --warmup 5 --audit-fraction $af > $O/audit_${af}.log 2>&1; rc=$?; ok $rc
  tail -1 $O/audit_${af}.log | cut -c1-200
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1; rc=$?; ok $rc
echo "prof rc=$rc"

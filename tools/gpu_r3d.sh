#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3d; mkdir -p $O
ok() { case $1 in 0|1) ;; *) echo "stop rc=$1"; exit $1 ;; esac; }
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k "audit_trail or edge_lines or pipeline_matches or overflow_chains or nan_elapsed or interleaved" > $O/k5_tests.log 2>&1; rc=$?
echo "k5 tests rc=$rc"; tail -2 $O/k5_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 60 --warmup 5 > $O/headline_$i.log 2>&1; rc=$?; ok $rc
  tail -1 $O/headline_$i.log | cut -c1-160
done
timeout -k 10 300 python bench.py --steps 60 --warmup 5 --audit-fraction 0.25 > $O/audit_0.25.log 2>&1; rc=$?; ok $rc
tail -1 $O/audit_0.25.log | cut -c1-160
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ser -o run -- python3 bench.py --steps 10 --warmup 3 --audit-fraction 0.25 > $O/ser.log 2>&1; rc=$?; ok $rc
echo "ser rc=$rc"

#!/bin/bash
# K5 / K1 check: (1) edge-corpus events with the host join (no device join kernels) == model;
# only then (2) the audit and edge tests through the device join, (3) bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/diag/k5_dump.py edge > gpurun_out/k5_edge.log 2>&1
rc=$?; echo "edge rc=$rc"; grep -v amdgpu.ids gpurun_out/k5_edge.log | tail -4
[ $rc -eq 0 ] || exit $rc
n=$(grep -c "extra \[\] missing \[\] fielddiff 0 " gpurun_out/k5_edge.log)
[ "$n" = "2" ] || { echo "edge events still differ: not running the device join on them"; exit 3; }
APM_DJ_DEBUG=1 timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_engine_gpu.py \
  -k "audit_trail or edge_lines" > gpurun_out/k5_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|debug|^E " gpurun_out/k5_tests.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/gpu_suite.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-300

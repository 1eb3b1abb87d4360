#!/bin/bash
# K5-on-device check: parse edge diff (diagnostic), the audit / join / checkpoint oracle tests,
# then the headline bench.  Each GPU step time-limited; stop at the first crash.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/diag/parse_edge_diff.py > gpurun_out/parse_diff.log 2>&1
rc=$?; echo "parse diff rc=$rc"; grep -E "^seed" gpurun_out/parse_diff.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_engine_gpu.py \
  -k "${K5_TESTS:-audit_trail or pipeline_matches_oracle or join_ or checkpoint or interleaved}" > gpurun_out/k5_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/k5_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-400

#!/bin/bash
# Where a checkpoint's ingest stall goes (service path, checkpoints on, stage trace) + the
# headline's kernel trace (blit copies by size).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ck; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py -k "grow_instead or checkpoint or audit_trail" > $O/ck_tests.log 2>&1; rc=$?
echo "ck tests rc=$rc"; tail -2 $O/ck_tests.log; [ $rc -eq 0 ] || exit $rc
D=$(mktemp -d -p "$PWD" svcdir.XXXX)
timeout -k 10 300 python bench.py --path service --service-dir "$D" --service-ckpt on --steps 200 --warmup 5 --trace $O/svc_trace.json > $O/svc.log 2>&1; rc=$?
rm -rf "$D"; echo "svc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/trace_summary.py $O/svc_trace.json > $O/svc_trace_summary.txt 2>&1
grep -E "ck\.|checkpoint" $O/svc_trace_summary.txt | head -20
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 bench.py --steps 10 --warmup 3 > $O/kt.log 2>&1; rc=$?
echo "kt rc=$rc"

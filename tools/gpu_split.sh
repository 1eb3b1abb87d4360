#!/bin/bash
# A/B: the st/fs D2H as two concurrent halves (default) vs one copy (APM_OUT_SPLIT=0), alternating,
# 60 steps; then the bench-scale oracle test (its fs text is large enough to be split).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/split; mkdir -p $O
for i in 1 2 3; do
  for v in 0 1; do
    APM_OUT_SPLIT=$v timeout -k 10 300 python bench.py --steps 60 --warmup 5 > $O/h_${v}_$i.log 2>&1 || exit $?
    python3 -c "
import json
d=json.loads([l for l in open('$O/h_${v}_$i.log') if l.startswith('{')][-1]); s=d['stage_ms_per_step']
print('split=$v', round(d['value']/1e6,1), d['ms_per_step'], 'join', s['t_join_ms'], 'out', s['t_out_ms'])"
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_scale_gpu.py tests/test_engine_gpu.py -k "headline_shard or sink_fds or pipeline_matches" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $O/tests.log

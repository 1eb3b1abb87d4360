#!/bin/bash
# Checkpoint path after the pinned-bounce / in-place snapshot change: checkpoint tests, then the
# service path with checkpoints off / on (alternating, 200 steps) and the stall breakdown.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ck2; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py tests/test_service_gpu.py -k "grow_instead or checkpoint or audit_trail or resume or service" > $O/ck_tests.log 2>&1; rc=$?
echo "ck tests rc=$rc"; tail -2 $O/ck_tests.log; [ $rc -eq 0 ] || exit $rc
D=$(mktemp -d -p "$PWD" svcdir.XXXX)
for ck in off on off on; do
  rm -rf "$D"/*
  f=$O/service_ckpt_${ck}_$RANDOM.log
  timeout -k 10 300 python bench.py --path service --service-dir "$D" --service-ckpt $ck --steps 200 --warmup 5 --trace $O/trace_$ck.json > $f 2>&1; rc=$?
  case $rc in 0|1) ;; *) rm -rf "$D"; exit $rc ;; esac
  python3 -c "
import json
d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); s=d['service']
ci=s.get('checkpoint_info') or {}
print('ckpt=$ck', round(d['value']/1e6,1), 'M lines/s; checkpoints', s.get('checkpoints'), {k: ci.get(k) for k in ('done','skipped','last_stall_ms','last_write_ms','last_bytes')})"
done
rm -rf "$D"
python3 - <<'PY'
import json
t=json.load(open('gpurun_out/ck2/trace_on.json'))
ev=t['traceEvents'] if isinstance(t,dict) else t
for e in ev:
    if e.get('name','').startswith('ck.'): print(e['name'], round(e.get('dur',0)/1000,2), 'ms')
PY

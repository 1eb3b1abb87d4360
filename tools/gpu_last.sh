#!/bin/bash
# Final tree check: GPU suite + smoke, st/fs D2H split A/B, service checkpoint A/B with spans.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/last; mkdir -p $O
ok() { case $1 in 0|1) ;; *) echo "stop rc=$1"; exit $1 ;; esac; }
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/gpu_suite.log 2>&1; rc=$?
echo "suite rc=$rc"; tail -2 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -1 $O/smoke.log; ok $rc
for i in 1 2; do
  for v in 0 1; do
    APM_OUT_SPLIT=$v timeout -k 10 300 python bench.py --steps 60 --warmup 5 > $O/split_${v}_$i.log 2>&1; rc=$?; ok $rc
    python3 -c "
import json
d=json.loads([l for l in open('$O/split_${v}_$i.log') if l.startswith('{')][-1]); s=d['stage_ms_per_step']
print('split=$v', round(d['value']/1e6,1), d['ms_per_step'], 'join', s['t_join_ms'], 'out', s['t_out_ms'])"
  done
done
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
print('ckpt=$ck', round(d['value']/1e6,1), 'M lines/s; checkpoints', s.get('checkpoints'), {k: ci.get(k) for k in ('done','last_stall_ms','last_bytes')})"
done
rm -rf "$D"
python3 - <<'PY'
import json
t=json.load(open('gpurun_out/last/trace_on.json'))
ev=t['traceEvents'] if isinstance(t,dict) else t
for e in ev:
    if e.get('name','').startswith('ck.'): print(e['name'], round(e.get('dur',0)/1000,2), 'ms')
PY

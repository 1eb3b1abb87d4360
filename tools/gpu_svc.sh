#!/bin/bash
# Production service path on the final tree: 200 steps, spool on the box's disk, fleet + lock-step,
# checkpoints on / off (alternating), firehose shard at 20/5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/svc; mkdir -p $O
D=$(mktemp -d -p "$PWD" svcdir.XXXX)
ok() { case $1 in 0|1) ;; *) echo "stop rc=$1"; rm -rf "$D"; exit $1 ;; esac; }
for ck in off on off on; do
  rm -rf "$D"/*
  timeout -k 10 300 python bench.py --path service --service-dir "$D" --service-ckpt $ck --steps 200 --warmup 5 > $O/service_ckpt_${ck}_$RANDOM.log 2>&1; rc=$?; ok $rc
  f=$(ls -t $O/service_ckpt_${ck}_*.log | head -1)
  python3 -c "
import json,sys
d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); s=d['service']
print('ckpt=$ck', round(d['value']/1e6,1), 'M lines/s; checkpoints', s.get('checkpoints'), 'info', {k: s['checkpoint_info'][k] for k in ('done','skipped','last_stall_ms','last_write_ms','last_bytes')} if s.get('checkpoint_info') else None, 'fs', s.get('fs_type'))"
done
rm -rf "$D"
timeout -k 10 420 python bench.py --preset firehose --steps 20 --warmup 5 > $O/firehose_20.log 2>&1; rc=$?; ok $rc
tail -1 $O/firehose_20.log | cut -c1-200

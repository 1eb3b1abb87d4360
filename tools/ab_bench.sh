#!/bin/bash
# A/B on one GPU box: alternate bench runs of the current tree and of a reference copy under
# ab/old (a previous build: cp -r apmbackend_amd bench.py profiles ab/old/), so box-to-box noise
# cancels.  Prints one "A|B value ms join stats" line per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:---steps 20 --warmup 3}
for i in $(seq ${ROUNDS:-3}); do
  for v in new old; do
    if [ $v = new ]; then d=.; else d=ab/old; fi
    (cd $d && timeout -k 10 300 python bench.py $ARGS > "$OLDPWD/gpurun_out/ab_${v}_$i.log" 2>&1)
    rc=$?
    if [ $rc -ne 0 ]; then echo "$v run $i rc=$rc"; tail -3 gpurun_out/ab_${v}_$i.log; exit $rc; fi
    python - "$v" "gpurun_out/ab_${v}_$i.log" <<'PY'
import json, sys
j = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
s = j["stage_ms_per_step"]
print(f"{sys.argv[1]:4s} {j['value']/1e6:7.2f}M lines/s {j['ms_per_step']:6.3f} ms  join {s['t_join_ms']:.3f} "
      f"shard {s.get('t_shard_busy_ms', 0):.3f} stats {s['t_stats_ms']:.3f}")
PY
  done
done

#!/bin/bash
# A/B of one build under two environments on one GPU box (box noise cancels by alternation):
#   A_ENV="APM_EVENTS_D2H=0" B_ENV="APM_EVENTS_D2H=1" ROUNDS=3 bash tools/ab_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:---steps 20 --warmup 3}
for i in $(seq ${ROUNDS:-3}); do
  for v in A B; do
    if [ $v = A ]; then e=${A_ENV:-}; else e=${B_ENV:-}; fi
    env $e timeout -k 10 300 python bench.py $ARGS > gpurun_out/abenv_${v}_$i.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$v run $i rc=$rc"; tail -3 gpurun_out/abenv_${v}_$i.log; exit $rc; fi
    python - "$v[$e]" "gpurun_out/abenv_${v}_$i.log" <<'PY'
import json, sys
j = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
s = j["stage_ms_per_step"]
print(f"{sys.argv[1]:24s} {j['value']/1e6:7.2f}M lines/s {j['ms_per_step']:6.3f} ms  parse {s['t_parse_ms']:.3f} join {s['t_join_ms']:.3f} "
      f"stats {s['t_stats_ms']:.3f} p50 {j['p50_ingest_to_alert_ms']:.2f}")
PY
  done
done

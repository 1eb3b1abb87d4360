#!/bin/bash
# Run-to-run spread of the 1-GPU headline bench with and without GPU-local thread pinning
# (alternating, so box drift hits both), plus the CPU topology the process is allowed to use.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
python - <<'PY' > gpurun_out/topo.txt 2>&1
import os
a = sorted(os.sched_getaffinity(0))
print("allowed", len(a), a[:64])
for c in a[:32]:
    p = f"/sys/devices/system/cpu/cpu{c}/topology/"
    sib = open(p + "thread_siblings_list").read().strip()
    core = open(p + "core_id").read().strip(); pkg = open(p + "physical_package_id").read().strip()
    print(c, "core", core, "pkg", pkg, "sib", sib)
PY
lscpu | grep -i "model name\|^L[23]\|NUMA\|Thread\|Socket" >> gpurun_out/topo.txt 2>&1 || true
for i in $(seq ${ROUNDS:-3}); do
  for pin in 0 1; do
    APM_PIN_THREADS=$pin timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/abpin_${pin}_$i.log 2>&1 || exit $?
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('pin=$pin', d['value'], d['ms_per_step'], d['pinned_cpus'], d.get('lane_cpus_head'), d['stage_ms_per_step']['t_join_ms'], d['stage_ms_per_step']['t_shard_max_ms'])" gpurun_out/abpin_${pin}_$i.log
  done
done

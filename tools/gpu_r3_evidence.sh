#!/bin/bash
# Round-3 evidence on one GPU: hardware counters of the hot kernels, a 200-step steady-state
# headline, the BASELINE configs, the audit-heavy shard (K5 host pre-pass) and the production
# service path with checkpoints on / off.  Every GPU step has its own limit; the script stops at
# the first failing step.  Usage: bash tools/gpu_r3_evidence.sh [pmc|bench|service|all]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3
mkdir -p $O
WHAT=${1:-all}
# heartbeat under gpurun_out/ (a long setup phase prints nothing for a while)
( while sleep 50; do date +%T >> $O/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
line() { tail -1 "$1" | cut -c1-200; }
run() {  # run NAME TIMEOUT ARGS...
  local n=$1 t=$2; shift 2
  echo "== $n: bench.py $*"
  timeout -k 10 "$t" python bench.py "$@" > $O/$n.log 2>&1 || { echo "$n failed rc=$?"; tail -5 $O/$n.log; exit 1; }
  line $O/$n.log
}
if [ "$WHAT" = pmc ] || [ "$WHAT" = all ]; then
  P="--steps 3 --warmup 1 --pre-batches 2"
  i=0
  for grp in "SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE TCC_HIT TCC_MISS" "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"; do
    i=$((i + 1))
    echo "== pmc pass $i: $grp"
    timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace --output-format csv --kernel-include-regex 'apm::' \
      -d $O/pmc/pmc$i -o run -- python3 bench.py $P > $O/pmc$i.log 2>&1 || { echo "pmc pass $i rc=$?"; tail -3 $O/pmc$i.log; exit 1; }
  done
  python tools/pmc_summary.py $O/pmc $O/pmc_kernels.md "rocprofv3 hardware counters, headline shard (round 3)"
  head -16 $O/pmc_kernels.md
fi
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
  run headline_200 600 --steps 200 --warmup 5
  run config2_60 300 --preset config2 --steps 60 --warmup 5
  run config4_60 300 --preset config4 --steps 60 --warmup 5
  run audit25_60 300 --audit-fraction 0.25 --steps 60 --warmup 5
  run audit02_60 300 --audit-fraction 0.02 --steps 60 --warmup 5
  run firehose_20 600 --preset firehose --steps 20 --warmup 5
  run firehose_60 600 --preset firehose --steps 60 --warmup 5
fi
if [ "$WHAT" = service ] || [ "$WHAT" = all ]; then
  run service_ckpt_on 900 --path service --steps 200 --warmup 5 --service-ckpt on
  run service_ckpt_off 900 --path service --steps 200 --warmup 5 --service-ckpt off
  run service_ckpt_on2 900 --path service --steps 200 --warmup 5 --service-ckpt on
fi
echo "evidence done"

#!/bin/bash
# MFMA A/B: K10 resync on matrix cores vs VALU, fleet moments by MFMA Gram pack vs fp64 atomic
# scatter.  Isolated kernel times (AMD_SERIALIZE_KERNEL=3 kernel trace) and whole-bench A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/mfma
mkdir -p $O
for v in mfma valu; do
  AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ser_$v -o run -- \
    python3 bench.py --steps 10 --warmup 3 --resync $v > $O/ser_$v.log 2>&1 || { echo "ser $v failed"; exit 1; }
  python tools/prof_summary.py $(ls $O/ser_$v/*kernel_stats.csv | head -1) $O/ks_$v.md "serialized kernels, --resync $v"
  echo "resync $v"; grep -E "resync|service_gram|k_zscore<" $O/ks_$v.md
done
APM_FLEET_ATOMIC=1 AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ser_atomic -o run -- \
  python3 bench.py --steps 10 --warmup 3 > $O/ser_atomic.log 2>&1 || { echo "ser atomic failed"; exit 1; }
python tools/prof_summary.py $(ls $O/ser_atomic/*kernel_stats.csv | head -1) $O/ks_atomic.md "serialized kernels, APM_FLEET_ATOMIC=1"
echo "fleet atomic"; grep -E "service_moments|service_gram" $O/ks_atomic.md
for i in 1 2; do
  for cfg in "--resync mfma" "--resync valu"; do
    timeout -k 10 300 python bench.py --steps 60 --warmup 5 $cfg > $O/ab.log 2>&1 || exit 1
    echo "$cfg: $(tail -1 $O/ab.log | cut -c1-110)"
  done
  for e in 0 1; do
    APM_FLEET_ATOMIC=$e timeout -k 10 300 python bench.py --steps 60 --warmup 5 > $O/ab.log 2>&1 || exit 1
    echo "APM_FLEET_ATOMIC=$e: $(tail -1 $O/ab.log | cut -c1-110)"
  done
done

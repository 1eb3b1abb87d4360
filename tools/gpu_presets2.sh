#!/bin/bash
# BASELINE config presets on the final tree (config2 bf16, config4 JMX fusion, firehose with the
# COPY spool through 4 writer lanes).  Each step time-limited; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/presets2
mkdir -p $O
for p in config2 config4 firehose; do
  timeout -k 10 420 python bench.py --preset $p --steps 10 --warmup 3 > $O/bench_$p.log 2>&1 || exit $?
  tail -1 $O/bench_$p.log | cut -c1-200
done
timeout -k 10 420 python bench.py --preset firehose --steps 10 --warmup 3 --writer-lanes 1 > $O/bench_firehose_l1.log 2>&1 || exit $?
tail -1 $O/bench_firehose_l1.log | cut -c1-200
echo done

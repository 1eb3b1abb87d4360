#!/bin/bash
# Headline performance evidence on one GPU: bench runs, host stage trace, kernel + copy timeline.
# Every GPU step has its own time limit; the script stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/perf
mkdir -p $O
for i in ${RUNS:-1 2}; do
  timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 > $O/headline_$i.log 2>&1 || exit $?
  tail -1 $O/headline_$i.log | cut -c1-240
done
timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --trace $O/trace.json > $O/bench_trace.log 2>&1 || exit $?
python tools/trace_summary.py $O/trace.json 38 > $O/trace_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tl -o run -- python3 bench.py --steps 12 --warmup 4 > $O/timeline.log 2>&1 || exit $?
python tools/gpu_timeline.py $O/tl --steps 10 > $O/timeline.txt
head -8 $O/timeline.txt
echo perf done

#!/bin/bash
# Presets + profile on one GPU (each step time-limited; stop at the first failure).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python bench.py --preset config2 --steps 10 --warmup 3 > gpurun_out/bench_config2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_config2.log
timeout -k 10 420 python bench.py --preset firehose --steps 10 --warmup 3 > gpurun_out/bench_firehose.log 2>&1 || exit $?
tail -1 gpurun_out/bench_firehose.log
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof.log 2>&1 || exit $?
echo prof done

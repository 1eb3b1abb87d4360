set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof.log 2>&1; rc=$?; echo "prof rc=$rc"; [ $rc -le 1 ] || exit $rc
for i in 1 2 3; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$i.log 2>&1; rc=$?; tail -1 gpurun_out/bench_$i.log | cut -c60-150; [ $rc -eq 0 ] || exit $rc
done

set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_$i.log 2>&1; rc=$?; tail -1 gpurun_out/bench_$i.log | cut -c60-150; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof2 -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof2.log 2>&1; echo "prof rc=$?"

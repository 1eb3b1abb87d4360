set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 200 --timeout-method thread -k "gram or fleet" > gpurun_out/t.log 2>&1; rc=$?; tail -6 gpurun_out/t.log; [ $rc -le 1 ] || exit $rc
for p in config4 firehose; do
timeout -k 10 400 python bench.py --preset $p --steps 10 --warmup 3 > gpurun_out/bench_$p.log 2>&1; rc=$?; echo "$p rc=$rc"; tail -1 gpurun_out/bench_$p.log | cut -c1-1500; [ $rc -le 1 ] || exit $rc
done

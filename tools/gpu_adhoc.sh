set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "rollup or oracle" > gpurun_out/t.log 2>&1; rc=$?; tail -3 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --preset config4 --steps 10 --warmup 3 > gpurun_out/bench_c4_$i.log 2>&1; rc=$?; tail -1 gpurun_out/bench_c4_$i.log | cut -c60-150; [ $rc -eq 0 ] || exit $rc
done

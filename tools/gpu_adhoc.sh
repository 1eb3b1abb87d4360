set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -1 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
for a in 1 0 1 0 1 0; do
APM_PULL_H2D=$a timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_ab.log 2>&1; rc=$?; echo "pull=$a $(tail -1 gpurun_out/bench_ab.log | cut -c60-150)"; [ $rc -eq 0 ] || exit $rc
done

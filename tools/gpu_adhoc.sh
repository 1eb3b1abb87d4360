set -u
mkdir -p gpurun_out
for a in 1 0 1 0 1 0; do
APM_DEFER_ROLLOVER=$a timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_ab.log 2>&1; rc=$?; echo "defer=$a $(tail -1 gpurun_out/bench_ab.log | cut -c60-150)"; [ $rc -eq 0 ] || exit $rc
done

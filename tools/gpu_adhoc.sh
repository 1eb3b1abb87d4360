set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_node_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_$i.log 2>&1; rc=$?; tail -1 gpurun_out/bench_$i.log | cut -c60-150; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --trace gpurun_out/mem_trace.json > gpurun_out/bench_tr.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
python tools/trace_summary.py gpurun_out/mem_trace.json | grep -v " u\."

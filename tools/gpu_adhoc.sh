set -u
mkdir -p gpurun_out/ev
for i in 1 2 3; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/ev/headline_$i.log 2>&1 || exit $?; tail -1 gpurun_out/ev/headline_$i.log | cut -c60-150
done
timeout -k 10 300 python bench.py --preset config2 --steps 20 --warmup 5 > gpurun_out/ev/config2.log 2>&1 || exit $?; tail -1 gpurun_out/ev/config2.log | cut -c60-150
timeout -k 10 420 python bench.py --preset firehose --steps 10 --warmup 3 --trace gpurun_out/ev/fh_trace.json > gpurun_out/ev/firehose.log 2>&1 || exit $?; tail -1 gpurun_out/ev/firehose.log | cut -c60-150
python tools/trace_summary.py gpurun_out/ev/fh_trace.json 5 | grep -v " u\." 

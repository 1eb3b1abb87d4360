set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_node_gpu.py tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread -k "fleet or gram or registry or node" > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --path service --steps 10 --warmup 3 > gpurun_out/svc_$i.log 2>&1 || exit $?
python - "$i" <<'P'
import json, sys
d = json.loads(open(f"gpurun_out/svc_{sys.argv[1]}.log").read().strip().splitlines()[-1])
s = d["service"]
print({k: s[k] for k in ("lines_per_s", "lines_per_s_engine_drained", "db_rows_per_s", "sink_write_ms", "seconds")})
P
done
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$i.log 2>&1; rc=$?; tail -1 gpurun_out/bench_$i.log | cut -c60-150; [ $rc -eq 0 ] || exit $rc
done

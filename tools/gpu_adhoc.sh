set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_service_gpu.py -x -v --timeout 200 --timeout-method thread -k "fs_copy or service" > gpurun_out/t.log 2>&1; rc=$?; tail -8 gpurun_out/t.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --path service --steps 10 --warmup 3 > gpurun_out/svc.log 2>&1; rc=$?; tail -1 gpurun_out/svc.log; [ $rc -le 1 ] || exit $rc

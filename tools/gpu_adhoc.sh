set -u
mkdir -p gpurun_out
for a in 1 0 1; do
APM_PREPASS_AHEAD=$a timeout -k 10 200 python -u -m pytest tests/test_service_gpu.py -x -q --timeout 100 --timeout-method thread -k readahead > gpurun_out/t_$a.log 2>&1; rc=$?; echo "ahead=$a rc=$rc"; grep "^E " gpurun_out/t_$a.log | head -8; [ $rc -le 1 ] || exit $rc
done

set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof.log 2>&1; rc=$?; echo "prof rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --kernel-trace --output-format csv --kernel-include-regex 'apm::' -d gpurun_out/pmc_mfma -o run -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/pmc_mfma.log 2>&1; rc=$?; echo "pmc rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --path service --steps 10 --warmup 3 --trace gpurun_out/svc_trace.json > gpurun_out/svc.log 2>&1; rc=$?; echo "svc rc=$rc"; tail -1 gpurun_out/svc.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --trace gpurun_out/mem_trace.json > gpurun_out/mem.log 2>&1; rc=$?; echo "mem rc=$rc"; tail -1 gpurun_out/mem.log

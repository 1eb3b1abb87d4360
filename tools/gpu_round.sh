#!/bin/bash
# Round evidence on one GPU: headline bench (x3), presets, service path, kernel stats, MFMA
# counters, host traces.  Each step time-limited; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/round
O=gpurun_out/round
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/headline_$i.log 2>&1 || exit $?
  tail -1 $O/headline_$i.log | cut -c1-160
done
for p in config2 config4 firehose; do
  timeout -k 10 420 python bench.py --preset $p --steps 10 --warmup 3 > $O/bench_$p.log 2>&1 || exit $?
  tail -1 $O/bench_$p.log | cut -c1-160
done
timeout -k 10 300 python bench.py --path service --steps 10 --warmup 3 --trace $O/svc_trace.json > $O/bench_service.log 2>&1 || exit $?
tail -1 $O/bench_service.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --trace $O/mem_trace.json > $O/bench_trace.log 2>&1 || exit $?
python tools/trace_summary.py $O/mem_trace.json > $O/mem_trace_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 3 > $O/prof.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --kernel-trace --output-format csv --kernel-include-regex 'apm::' -d $O/pmc_mfma -o run -- python3 bench.py --steps 3 --warmup 1 > $O/pmc_mfma.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv --kernel-include-regex 'apm::' -d $O/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 > $O/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT TCC_MISS --kernel-trace --output-format csv --kernel-include-regex 'apm::' -d $O/pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 > $O/pmc_write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-trace --output-format csv --kernel-include-regex 'apm::' -d $O/pmc_lds -o run -- python3 bench.py --steps 3 --warmup 1 > $O/pmc_lds.log 2>&1 || exit $?
echo all done

#!/bin/bash
# GPU-box check used through gpurun: tests -> smoke -> bench -> optional rocprof.
# Each GPU step has its own time limit; after a crash/abort/timeout nothing else touches the GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
stop_on_fault() {  # $1 = rc, $2 = step name
  case "$1" in
    0|1) return 0 ;;
    *) echo "GPU step $2 ended with rc=$1 -- stopping (no further GPU work)"; exit "$1" ;;
  esac
}
STEPS="${STEPS:-tests smoke bench}"
for s in $STEPS; do
  case "$s" in
    tests)
      timeout -k 10 "${T_TESTS:-420}" python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/tests.log 2>&1
      rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/tests.log; stop_on_fault $rc tests ;;
    smoke)
      timeout -k 10 "${T_SMOKE:-240}" python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; stop_on_fault $rc smoke ;;
    bench)
      timeout -k 10 "${T_BENCH:-420}" python bench.py ${BENCH_ARGS:---steps 10 --warmup 3} > gpurun_out/bench.log 2>&1
      rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log; stop_on_fault $rc bench ;;
    prof)
      timeout -k 10 "${T_PROF:-420}" rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py ${PROF_ARGS:---steps 5 --warmup 2} > gpurun_out/prof.log 2>&1
      rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/prof.log; stop_on_fault $rc prof ;;
    pmc)
      # hardware counters of the engine's own kernels, one rocprofv3 pass per counter group
      # (per-block limits: <= 8 SQ, <= 4 TCC -- FETCH_SIZE takes 3, WRITE_SIZE 2)
      i=0
      for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
                 "FETCH_SIZE TCP_TOTAL_CACHE_ACCESSES_sum" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" \
                 "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM"; do
        i=$((i+1))
        timeout -s KILL "${T_PMC:-120}" rocprofv3 --pmc $grp --kernel-trace --output-format csv --kernel-include-regex 'apm::' \
          -d gpurun_out/pmc$i -o run -- python3 bench.py ${PMC_ARGS:---steps 3 --warmup 1} > gpurun_out/pmc$i.log 2>&1
        rc=$?; echo "pmc pass $i rc=$rc"; tail -2 gpurun_out/pmc$i.log; stop_on_fault $rc pmc$i
      done ;;
  esac
done

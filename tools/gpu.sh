#!/bin/bash
# One parameterised GPU-box runner (replaces the round-1..3 one-off gpu_*.sh scripts).
#
#   gpurun --timeout 1200 -- 'bash tools/gpu.sh OUT TASK [TASK ...]'
#
# OUT is a directory under gpurun_out/ (copied back by gpurun); every task writes its log there,
# and the profile directories under profiles/ name the task list that produced them.  Every GPU
# step runs under its own `timeout -k 10`; the script stops at the first step that crashes,
# aborts or times out (no retries).
#
# Tasks:
#   suite              pytest -m gpu (thread-method timeouts, stops at the first failure)
#   suite:EXPR         pytest -m gpu -k EXPR
#   suiteall:EXPR      the same without stopping at the first failure
#   smoke              __graft_entry__.smoke()
#   bench[:STEPS]      driver-shaped bench.py (warmup 5), default 20 steps
#   bench200           200-step headline (steady state)
#   ranks:N            torchrun N ranks of bench.py on the one GPU (host transport), rank reports
#   preset:NAME        bench.py --preset NAME (config2, config4, firehose) 20/5
#   service            bench.py --path service (production path, checkpoints on), 200 steps
#   prof               rocprofv3 --kernel-trace --stats of bench.py 20/5
#   trace              bench.py 60/5 with the engine's Chrome trace (tools/trace_summary.py reads it)
#   profser            the same with every kernel serialised (AMD_SERIALIZE_KERNEL=3): isolated kernel times
#   timeline           rocprofv3 --kernel-trace --memory-copy-trace (tools/gpu_timeline.py reads it)
#   pmc:C1,C2,...      one rocprofv3 --pmc pass of bench.py 10/3 (keep within one pass's counter budget)
#   service:T          the same with T tailer read threads
#   servicetrace       the service path with the engine's Chrome trace
#   servicex:A,B       the service path with extra bench.py arguments A B
#   benchx:A,B         bench.py 20/5 with extra arguments A B (commas become spaces)
#   benchold           bench.py 20/5 of the copy under ab/old (a previous tree's package + build,
#                      shipped by taking ./ab out of .gpurunignore for that call): same-box A/B
#   meminfo            append the page cache's dirty / writeback counters and the vm.dirty_*
#                      limits to OUT/meminfo.log (service-path spread attribution)
#   sync               flush dirty pages to disk (sync) and log how long it took
#   env:K=V            export K=V for the following tasks (A/B switches; BENCH_EXTRA=--a=b adds
#                      bench.py arguments to the profser / pmc runs)
#   unenv:K            unset K for the following tasks
#   py:MODULE          python -m MODULE (diagnostics under tools/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:?usage: gpu.sh OUT TASK...}
shift
mkdir -p "$O"
stop() { echo "STOP: $1 rc=$2"; exit "$2"; }
run() {  # run NAME SECONDS CMD...
  local name=$1 secs=$2
  shift 2
  local t0=$(date +%s)
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc $(( $(date +%s) - t0 ))s :: $(tail -c 600 "$O/$name.log" | tail -n 2 | cut -c1-400)"
  # pytest rc 1 = assertion failures only (no fault, no hang: a timeout or a crash ends the run)
  if [ $rc -eq 1 ] && [[ $name == suite* ]] && ! grep -qE "Timeout|Fatal Python error|core dumped|HSA_STATUS|Memory access fault" "$O/$name.log"; then
    echo "[$name] test failures (no fault): continuing"; return 0
  fi
  case $rc in 0) ;; *) stop "$name" $rc ;; esac
}
n=0
for task in "$@"; do
  n=$((n + 1))
  case $task in
    suite) run "suite" 1100 python -u -m pytest --maxfail 6 -v --timeout 240 --timeout-method thread tests -m gpu ;;
    suiteall:*) run "suite_$n" 1000 python -u -m pytest --maxfail 10 -v --timeout 240 --timeout-method thread tests -m gpu -k "${task#suiteall:}" ;;
    suite:*) run "suite_$n" 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests -m gpu -k "${task#suite:}" ;;
    smoke) run "smoke" 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run "bench_$n" 300 python -u bench.py --steps 20 --warmup 5 ;;
    bench:*) run "bench_$n" 400 python -u bench.py --steps "${task#bench:}" --warmup 5 ;;
    benchold) run "benchold_$n" 300 bash -c "cd ab/old && python -u bench.py --steps 20 --warmup 5" ;;
    benchx:*) a=${task#benchx:}; run "benchx_$n" 300 python -u bench.py --steps 20 --warmup 5 ${a//,/ } ;;
    bench200) run "bench200_$n" 400 python -u bench.py --steps 200 --warmup 5 ;;
    ranks:*)
      w=${task#ranks:}
      run "ranks${w}_$n" 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node="$w" \
        --master-addr=127.0.0.1 --master-port=$((29400 + n)) bench.py --gpus "$w" --steps 40 --warmup 5 \
        --rank-report "$O/ranks${w}_$n" ;;
    preset:*) run "preset_${task#preset:}_$n" 500 python -u bench.py --preset "${task#preset:}" --steps 20 --warmup 5 ;;
    service) run "service_$n" 600 python -u bench.py --path service --steps 200 --warmup 5 --service-dir /tmp/apm_svc ;;
    servicex:*) a=${task#servicex:}; run "servicex_$n" 600 python -u bench.py --path service --steps 200 --warmup 5 \
                  --service-dir /tmp/apm_svc ${a//,/ } ;;
    servicetrace) run "servicetrace_$n" 600 python -u bench.py --path service --steps 200 --warmup 5 \
                    --service-dir /tmp/apm_svc --trace "$O/servicetrace_$n.json" ;;
    service:*) run "service${task#service:}_$n" 600 python -u bench.py --path service --steps 200 --warmup 5 \
                 --service-dir /tmp/apm_svc --tail-read-threads "${task#service:}" ;;
    prof) run "prof_$n" 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$n" -o run -- \
            python3 bench.py --steps 20 --warmup 5 ;;
    trace) run "trace_$n" 300 python -u bench.py --steps 60 --warmup 5 --trace "$O/trace_$n.json" ;;
    profser) AMD_SERIALIZE_KERNEL=3 run "profser_$n" 600 rocprofv3 --kernel-trace --stats --output-format csv \
               -d "$O/profser_$n" -o run -- python3 bench.py --steps 10 --warmup 3 ${BENCH_EXTRA:-} ;;
    timeline) run "timeline_$n" 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$O/tl_$n" -o run -- \
                python3 bench.py --steps 20 --warmup 5 ;;
    pmc:*) c=${task#pmc:}; run "pmc_$n" 120 rocprofv3 --kernel-trace --pmc ${c//,/ } --output-format csv -d "$O/pmc_$n" -o run -- \
             python3 bench.py --steps 10 --warmup 3 ${BENCH_EXTRA:-} ;;
    meminfo) { echo "[$n] $(date +%T.%N)"; grep -E '^(Dirty|Writeback|MemFree|Cached):' /proc/meminfo | tr -s ' ' | tr '\n' ' ';
               echo; for f in dirty_ratio dirty_background_ratio dirty_bytes dirty_background_bytes dirty_expire_centisecs; do
               echo -n "$f=$(cat /proc/sys/vm/$f 2>/dev/null) "; done; echo; df -h /tmp | tail -1; echo "loadavg $(cat /proc/loadavg)";
               for r in cpu memory io; do echo "psi.$r $(tr '\n' ' ' < /proc/pressure/$r 2>/dev/null)"; done; } >> "$O/meminfo.log" ;;
    sync) t0=$(date +%s%N); timeout -k 10 300 sync; rc=$?; echo "[$n] sync rc=$rc $(( ($(date +%s%N) - t0) / 1000000 )) ms" | tee -a "$O/meminfo.log" ;;
    env:*) export "${task#env:}"; echo "[env] ${task#env:}" ;;
    unenv:*) unset "${task#unenv:}"; echo "[unenv] ${task#unenv:}" ;;
    py:*) run "py_$n" 600 python -u -m "${task#py:}" "$O" ;;
    *) echo "unknown task $task"; exit 2 ;;
  esac
done
echo "ALL OK"

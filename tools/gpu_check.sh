#!/usr/bin/env bash
# One GPU-box session: smoke -> GPU tests -> bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; a crash/abort/timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
stop_if_fatal() {  # $1 = rc, $2 = step; pytest rc 1 = test failures (not fatal)
  case "$1" in
    0) ;;
    1) [ "$2" = pytest ] || { echo "step $2 failed rc=$1"; exit "$1"; } ;;
    *) echo "step $2 fatal rc=$1 -- stopping"; exit "$1" ;;
  esac
}
STEPS="${STEPS:-smoke pytest bench prof}"
for s in $STEPS; do
  echo "== $s $(date +%T)"
  case "$s" in
    smoke)  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$? ;;
    pytest) timeout -k 10 1200 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
              --durations=15 ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1; rc=$? ;;
    bench)  # the driver's own command line (BENCH_rNN.json)
            timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$? ;;
    benchall)  # every BASELINE config, each with its CPU baseline
      rc=0
      for c in ${CFGS:-1 2 3 4 5}; do
        timeout -k 10 600 python3 bench.py --workload cfg$c --steps 20 > "$OUT/bench_cfg$c.json" \
          2> "$OUT/bench_cfg$c.err" || { rc=$?; break; }
        tail -1 "$OUT/bench_cfg$c.json"
      done ;;
    prof)   timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
              python3 bench.py --steps 20 --no-cpu > "$OUT/prof_bench.json" 2> "$OUT/prof.err"; rc=$? ;;
    sweep)  timeout -k 10 900 python3 tools/sweep.py ${SWEEP_ARGS:-} > "$OUT/sweep.jsonl" 2> "$OUT/sweep.err"; rc=$? ;;
    *) echo "unknown step $s"; rc=0 ;;
  esac
  echo "   rc=$rc"
  case "$s" in pytest) f=pytest_gpu.log ;; smoke) f=smoke.log ;; bench) f=bench.json ;; sweep) f=sweep.err ;;
    benchall) f=/dev/null ;; *) f=prof.err ;; esac
  tail -3 "$OUT/$f" 2>/dev/null
  stop_if_fatal "$rc" "$s"
done
echo "== done $(date +%T)"

#!/usr/bin/env bash
# rocprofv3 passes over the headline bench (run on the GPU box):
#   1. --kernel-trace --stats      per-kernel durations (must agree with bench.py's HIP-event timing)
#   2. --pmc FETCH_SIZE            HBM read bytes per dispatch (KB; gfx950 reports 1/2 of wide streams)
#   3. --pmc WRITE_SIZE            HBM write bytes per dispatch (KB)
# Counters go in their own passes, never combined with sys/runtime tracing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG="${TAG:-r01}"
WL="${WL:-cfg5}"
OUT="gpurun_out/prof_${TAG}_${WL}"
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH_ARGS="--workload $WL --no-cpu ${PKTS:+--packets-per-gpu $PKTS}"
run() {  # $1 = name, rest = rocprofv3 args
  local name=$1; shift
  echo "== $name $(date +%T)"
  timeout -k 10 600 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv -- \
    python3 bench.py $BENCH_ARGS > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?
  echo "   rc=$rc"; tail -2 "$OUT/$name.err"
  [ $rc -eq 0 ] || exit $rc
}
run trace --kernel-trace --stats  # bench defaults: 20 steps, 40 warmup
BENCH_ARGS="$BENCH_ARGS --steps 3 --warmup 1"
run pmc_fetch --pmc FETCH_SIZE
run pmc_write --pmc WRITE_SIZE
python3 tools/prof_summary.py "$OUT" "$TAG" "$WL" || true  # condensed again on the build host after the merge

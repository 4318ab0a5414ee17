#!/usr/bin/env bash
# End-of-round evidence on one GPU box: smoke, GPU tests, a bench line per
# BASELINE config (each with its CPU baseline), then the rocprofv3 passes of
# tools/prof_all.sh (trace + FETCH + WRITE per config, SQ counters for
# cfg2/cfg4).  Every GPU step has its own time limit; the first failure stops.
#   TAG=r02b bash tools/round_final.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TAG="${TAG:-r02}"
STEPS="smoke pytest benchall" bash tools/gpu_check.sh || exit $?
mkdir -p gpurun_out/final_${TAG}
cp gpurun_out/bench_cfg*.json gpurun_out/final_${TAG}/ 2>/dev/null
bash tools/prof_all.sh || exit $?
echo "== round_final done $(date +%T)"

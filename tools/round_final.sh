#!/usr/bin/env bash
# End-of-round evidence on one GPU box: smoke, GPU tests, then the rocprofv3
# passes of tools/prof_all.sh (trace + FETCH + WRITE per config, SQ counters
# for cfg2/cfg4) -- whose summaries rewrite profiles/traffic_<cfg>.json on the
# box -- and only then a bench line per BASELINE config (each with its CPU
# baseline), so every line's roofline.traffic comes from a PMC pass over the
# same kernel of the same build.  Every GPU step has its own time limit; the
# first failure stops.  After the merge, rerun tools/prof_summary.py here on
# gpurun_out/prof_<TAG>_<cfg> (same inputs, same traffic files).
#   TAG=r03 bash tools/round_final.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TAG="${TAG:-r03}"
STEPS="smoke pytest" bash tools/gpu_check.sh || exit $?
bash tools/prof_all.sh || exit $?
STEPS="benchall" bash tools/gpu_check.sh || exit $?
mkdir -p gpurun_out/final_${TAG}
cp gpurun_out/bench_cfg*.json gpurun_out/final_${TAG}/ 2>/dev/null
echo "== round_final done $(date +%T)"

#!/usr/bin/env bash
# End-of-round-6 evidence on the final build, in phases that each fit one
# gpurun call (limit 20 min); every GPU step has its own time limit and the
# first failure stops the phase.  After each merge, rerun tools/prof_summary.py /
# tools/pmc_rx_summary.py here on the merged gpurun_out (same inputs).
#   PHASE=1 bash tools/r06_final.sh   smoke, GPU tests, rocprof + PMC for cfg1 (256M, 1M), cfg2, cfg3
#   PHASE=2 bash tools/r06_final.sh   rocprof + PMC for cfg4, cfg5; SQ counters for cfg4
#   PHASE=3 bash tools/r06_final.sh   a bench line per BASELINE config, each with its CPU baseline
#   PHASE=4 bash tools/r06_final.sh   RX: PMC passes, the ring schedules, the byte-packed verifier
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TAG="${TAG:-r06}"
mkdir -p gpurun_out
case "${PHASE:-1}" in
  1) STEPS="smoke pytest" bash tools/gpu_check.sh || exit $?
     WLS="cfg1:268435456 cfg1 cfg2 cfg3" SQ_WLS=" " bash tools/prof_all.sh || exit $? ;;
  2) WLS="cfg4 cfg5" SQ_WLS="cfg4" bash tools/prof_all.sh || exit $? ;;
  3) STEPS="benchall" bash tools/gpu_check.sh || exit $?
     mkdir -p gpurun_out/final_${TAG} && cp gpurun_out/bench_cfg*.json gpurun_out/final_${TAG}/ ;;
  4) TAG=$TAG bash tools/pmc_rx.sh > gpurun_out/pmc_rx_${TAG}.log 2>&1 || { echo "pmc_rx failed"; tail -20 gpurun_out/pmc_rx_${TAG}.log; exit 1; }
     timeout -k 10 900 python3 tools/rx_device_bench.py --rounds 3 > gpurun_out/rx_device_${TAG}.jsonl \
       2> gpurun_out/rx_device_${TAG}.err || { echo "rx bench rc=$?"; exit 1; } ;;
esac
echo "== phase ${PHASE:-1} done $(date +%T)"

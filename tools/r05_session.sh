#!/usr/bin/env bash
# Round-5 GPU sessions (one box per call), steps chosen by STEPS:
#   ring    the RX ring schedules A/B (tools/rx_device_bench.py, 3 rounds)
#   probe   cfg4's ceiling: loads-only streams over cfg4's 8.27 GB and cfg3's
#           9.4 GB (k_packedb's and k_flat_coop's schedules), then the cfg4 bench
#   pmcrx   tools/pmc_rx.sh (FETCH/WRITE per RX workload)
# Every GPU step has its own limit; the first failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
TAG="${TAG:-r05}"
for s in ${STEPS:-ring}; do
  echo "== $s $(date +%T)"
  case "$s" in
    ringab) T=$(python3 -c "import json;print(','.join('groups:'+k for k in json.load(open('tools/ring_tunes_r05.json'))))")
           timeout -k 10 600 python3 tools/rx_device_bench.py --skip-packed --rounds 2 --arms "groups,rows,slots,$T" \
             --tunes "$(cat tools/ring_tunes_r05.json)" > "$OUT/ringab_${TAG}.jsonl" 2> "$OUT/ringab_${TAG}.err" \
             || { echo "ringab rc=$?"; tail -5 "$OUT/ringab_${TAG}.err"; exit 1; } ;;
    ringtest) timeout -k 10 400 python3 -u -m pytest tests/test_gpu_bounds.py tests/test_gpu_rx.py -k ring -m gpu -x -q \
             --timeout 300 --timeout-method thread > "$OUT/ringtest_${TAG}.log" 2>&1 || { echo "ringtest failed"; tail -20 "$OUT/ringtest_${TAG}.log"; exit 1; }
           tail -1 "$OUT/ringtest_${TAG}.log" ;;
    ring)  timeout -k 10 600 python3 tools/rx_device_bench.py --skip-packed --rounds 3 \
             > "$OUT/ring_${TAG}.jsonl" 2> "$OUT/ring_${TAG}.err" || { echo "ring rc=$?"; tail -5 "$OUT/ring_${TAG}.err"; exit 1; } ;;
    probe) PROBE_ARMS=disp_u32_w1_t64,disp_u32_w1_t128,disp_u24_w4_t64,coop_u32_w4_t64,coop_u24_w4_t64 \
             timeout -k 10 200 pip_amd/lib/stream_probe 8.275,9.4 3 > "$OUT/probe_${TAG}.jsonl" 2> "$OUT/probe_${TAG}.err" \
             || { echo "probe rc=$?"; exit 1; }
           timeout -k 10 300 python3 bench.py --workload cfg4 --no-cpu > "$OUT/bench_cfg4_${TAG}.json" \
             2> "$OUT/bench_cfg4_${TAG}.err" || { echo "bench rc=$?"; exit 1; } ;;
    pytest) timeout -k 10 1200 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
             > "$OUT/pytest_${TAG}.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_${TAG}.log"; exit 1; }
           tail -1 "$OUT/pytest_${TAG}.log" ;;
    pmcrx) TAG=$TAG bash tools/pmc_rx.sh > "$OUT/pmc_rx_${TAG}.log" 2>&1 || { echo "pmcrx failed"; exit 1; } ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "== done $(date +%T)"

#!/usr/bin/env bash
# rocprofv3 passes over the RX verifiers, on the GPU box:
# for each workload of tools/rx_device_bench.py -- the byte-packed frames
# (k_packedb_rx, pipck_rx_verify_device) and the rings (k_ring, the default of
# pipck_rx_verify_ring) -- a kernel trace, a FETCH_SIZE pass and a WRITE_SIZE
# pass, each its own process (counters never combined with other tracing).
# tools/pmc_rx_summary.py then writes profiles/traffic_rx_<workload>.json.
#   TAG=r05 bash tools/pmc_rx.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG="${TAG:-r05}"
export TMPDIR=/tmp
for wl in ${RX_WLS:-packed ring_sparse_9216 ring_dense_1536 ring_dense_9216 ring_short_2048 ring_short_1024}; do
  OUT="gpurun_out/pmc_rx_${TAG}_${wl}"
  mkdir -p "$OUT"
  if [ "$wl" = packed ]; then ARGS="--rings none --rounds 1"; else ARGS="--skip-packed --rings $wl --arms groups --rounds 1"; fi
  for pass in trace pmc_fetch pmc_write; do
    case $pass in
      trace) P="--kernel-trace --stats"; IT="--iters 10 --warm 10" ;;
      pmc_fetch) P="--pmc FETCH_SIZE"; IT="--iters 3 --warm 1" ;;
      pmc_write) P="--pmc WRITE_SIZE"; IT="--iters 3 --warm 1" ;;
    esac
    echo "== $wl $pass $(date +%T)"
    timeout -k 10 400 rocprofv3 $P -d "$OUT/$pass" -o run --output-format csv -- \
      python3 tools/rx_device_bench.py $ARGS $IT > "$OUT/$pass.jsonl" 2> "$OUT/$pass.err"
    rc=$?
    echo "   rc=$rc"
    [ $rc -eq 0 ] || { tail -5 "$OUT/$pass.err"; exit $rc; }
  done
done
python3 tools/pmc_rx_summary.py "$TAG" || true  # condensed again on the build host after the merge
echo "== pmc_rx done"

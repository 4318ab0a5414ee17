#!/usr/bin/env bash
# VERDICT r03 item 6 on one box: the k_hdr result-stream A/B at 256M headers,
# then per arm one rocprofv3 pass each for FETCH_SIZE, WRITE_SIZE and the SQ
# stall counters.  Run it in two gpurun calls (two boxes) and compare.
#   TAG=boxA bash tools/hdr_spread.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG="${TAG:-box}"
OUT="gpurun_out/hdr_spread_$TAG"
mkdir -p "$OUT"
timeout -k 10 300 python3 tools/hdr_spread.py > "$OUT/ab.jsonl" 2> "$OUT/ab.err" || { tail -5 "$OUT/ab.err"; exit 1; }
cat "$OUT/ab.jsonl"
for arm in default in_place; do
  for c in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU"; do
    tag=$(echo "$c" | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $c -d "$OUT/${arm}_$tag" -o run --output-format csv -- \
      python3 tools/hdr_spread.py --pmc-arm "$arm" > /dev/null 2> "$OUT/${arm}_$tag.err" || { echo "pmc $arm $tag rc=$?"; exit 1; }
  done
done
echo "== hdr_spread $TAG done"

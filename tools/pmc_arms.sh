#!/usr/bin/env bash
# FETCH_SIZE / WRITE_SIZE per dispatch for size_scan arms, one rocprofv3 pass per
# (arm, counter); then a one-line summary per arm (HBM bytes per launch, gfx950
# correction: 2 x FETCH_SIZE).
#   ONLY=cfg4 SIZES=8 EXTRA=--packed ARMS='{"a": {}, "b": {...}}' bash tools/pmc_arms.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_arms
mkdir -p "$OUT"
python3 - "$ARMS" > "$OUT/arm_names.txt" <<'PY'
import json, sys
for k in json.loads(sys.argv[1]): print(k)
PY
while read -r arm; do
  spec=$(python3 -c 'import json,sys; a=json.loads(sys.argv[1]); print(json.dumps({sys.argv[2]: a[sys.argv[2]]}))' "$ARMS" "$arm")
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c -d "$OUT/${arm}_$c" -o run --output-format csv -- \
      python3 tools/size_scan.py --only "$ONLY" --sizes "$SIZES" --iters 3 ${EXTRA:-} --arms "$spec" \
      > "$OUT/${arm}_$c.jsonl" 2> "$OUT/${arm}_$c.err" || exit $?
  done
done < "$OUT/arm_names.txt"
echo "== pmc_arms done"

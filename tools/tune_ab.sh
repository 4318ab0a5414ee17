# bench.py's own line under engine.tune arms (TUNES: space-separated JSON
# objects, '{}' = the default), one process per (round, arm), arms alternating;
# WL (default cfg5), ROUNDS (default 2).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-tune_ab}.jsonl
: > "$OUT"
for r in $(seq 1 "${ROUNDS:-2}"); do
  for t in ${TUNES:-'{}'}; do
    timeout -k 10 200 python3 bench.py --workload "${WL:-cfg5}" --no-cpu --tune "$t" > gpurun_out/tab_one.json 2>> gpurun_out/tune_ab.err || exit 1
    python3 -c "
import json, sys; d=json.loads(open('gpurun_out/tab_one.json').read().strip().splitlines()[-1]); r=d['roofline']
print(json.dumps({'round': $r, 'tune': json.loads(sys.argv[1]), 'workload': '${WL:-cfg5}', 'kernel': r['kernel'].split('(')[0], 'kernel_ms': r['kernel_ms'], 'frac': r['frac']}))" "$t" >> "$OUT"
  done
done
cat "$OUT"

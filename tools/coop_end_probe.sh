# MEASUREMENT ONLY: where k_flat_coop's time goes on cfg2 / cfg3 / cfg5 --
# the production kernel, the same stream with no task end (tune bit 22: no
# results) and loads only (bit 21: every row consumed with one add), one box,
# rounds interleaved.  One JSON line per (round, workload, arm).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
: > gpurun_out/coop_end_probe.jsonl
for r in 1 2; do
  for c in cfg2 cfg3 cfg5; do
    for t in '{}' '{"no_task_end": true}' '{"loads_only": true}'; do
      timeout -k 10 200 python3 bench.py --workload $c --no-cpu --tune "$t" > gpurun_out/cep_one.json 2>> gpurun_out/coop_end_probe.err || exit 1
      python3 -c "
import json, sys; d=json.loads(open('gpurun_out/cep_one.json').read().strip().splitlines()[-1]); r=d['roofline']
print(json.dumps({'round': $r, 'workload': '$c', 'tune': json.loads(sys.argv[1]), 'kernel': r['kernel'].split('(')[0], 'kernel_ms': r['kernel_ms'], 'frac': r['frac']}))" "$t" >> gpurun_out/coop_end_probe.jsonl
    done
  done
done
cat gpurun_out/coop_end_probe.jsonl

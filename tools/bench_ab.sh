# bench.py's own cfgN line under several libpipck builds (PIPCK_LIB), one
# process per (round, build), builds alternating: ARMS="name=path ..." (cur =
# pip_amd/lib/libpipck.so), WL (default cfg2), ROUNDS (default 4).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-bench_ab}.jsonl
: > "$OUT"
for r in $(seq 1 "${ROUNDS:-4}"); do
  for arm in ${ARMS:-cur=pip_amd/lib/libpipck.so}; do
    name=${arm%%=*}; lib=${arm#*=}
    PIPCK_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --workload "${WL:-cfg2}" --no-cpu > gpurun_out/bab_one.json 2>> gpurun_out/bench_ab.err || exit 1
    python3 -c "
import json, sys; d=json.loads(open('gpurun_out/bab_one.json').read().strip().splitlines()[-1]); r=d['roofline']
print(json.dumps({'round': $r, 'arm': sys.argv[1], 'workload': '${WL:-cfg2}', 'kernel_ms': r['kernel_ms'], 'b2b_ms': r['kernel_ms_b2b_mean'], 'frac': r['frac'], 'lib': r['lib_sha256'][:12]}))" "$name" >> "$OUT"
  done
done
cat "$OUT"

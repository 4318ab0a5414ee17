# k_ring against a measurement-only build of itself that streams the same
# loads with no per-slot work and no parse (pip_amd/lib/ab/libpipck_ringlo.so):
# every ring, one process per (round, build).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
OUT=gpurun_out/ring_ceiling.jsonl
: > "$OUT"
for r in 1 2; do
  for arm in cur=pip_amd/lib/libpipck.so lo=pip_amd/lib/ab/libpipck_ringlo.so; do
    name=${arm%%=*}; lib=${arm#*=}
    PIPCK_LIB=$PWD/$lib timeout -k 10 400 python3 tools/rx_device_bench.py --skip-packed --rounds 1 --arms groups \
      > gpurun_out/rc_one.jsonl 2>> gpurun_out/ring_ceiling.err || exit 1
    python3 -c "
import json, sys
for l in open('gpurun_out/rc_one.jsonl'):
    d = json.loads(l); print(json.dumps({'round': $r, 'build': sys.argv[1], 'ring': d['what'], 'ms': d['ms'], 'frac': d['frac']}))" "$name" >> "$OUT"
  done
done
cat "$OUT"

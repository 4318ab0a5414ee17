set -u
cd "${GRAFT_REPO_ROOT:-.}"
: > gpurun_out/rx_ab.jsonl
for r in 1 2; do
for t in '{"loads_per_lane": 48}' '{"loads_per_lane": 46}' '{"loads_per_lane": 24}' '{"loads_per_lane": 28}' '{"loads_per_lane": 32}'; do
  timeout -k 10 300 python3 tools/rx_device_bench.py --rings none --rounds 2 --tune "$t" >> gpurun_out/rx_ab.jsonl 2>> gpurun_out/rx_ab.err || exit 1
done
done
grep rx_verify_device gpurun_out/rx_ab.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['last_kernel'], d['ms'], d['frac'])"

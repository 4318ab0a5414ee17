# k_packedb_rx's block shapes on the 8M-frame batch (tools/rx_device_bench.py,
# packed arms only): tune loads_per_lane {} = the default 4 waves x ring 8,
# 28 = 2 x 16, 32 = 1 x 32 (the round-4 kernel).  The wider sweep behind the
# default (4 x 6, 2 x 8, 8 x 2..6) ran on shapes since removed from the
# launcher (profiles/r05_packedb_rx_waves_explore.jsonl).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
: > gpurun_out/rx_ab.jsonl
for r in 1 2; do
for t in '{}' '{"loads_per_lane": 28}' '{"loads_per_lane": 32}'; do
  timeout -k 10 300 python3 tools/rx_device_bench.py --rings none --rounds 2 --tune "$t" >> gpurun_out/rx_ab.jsonl 2>> gpurun_out/rx_ab.err || exit 1
done
done
grep rx_verify_device gpurun_out/rx_ab.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['last_kernel'], d['ms'], d['frac'])"

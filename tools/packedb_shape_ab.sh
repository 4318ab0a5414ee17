# k_packedb's block width / ring depth A/B on one box: the byte-packed parity
# tests (every shape), then cfg4's bench line and the RX device verifier per
# shape (internal tune loads_per_lane: 0 = the defaults, k_packedb 8 waves with a ring of 3 and k_packedb_rx 4 with 8;
# 32 = one wave, ring 32; 48 = 4 waves, ring 8; 72 / 74 = 8 waves, ring 2 / 4; RX: 28 = 2 waves, ring 16).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rx.py -k "packed_bytes or packedb or rx_verify_device" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_pb4.log 2>&1 || { tail -30 gpurun_out/pytest_pb4.log; exit 1; }
tail -1 gpurun_out/pytest_pb4.log
: > gpurun_out/pb4_ab.jsonl
for r in 1 2; do
  for t in '{}' '{"loads_per_lane": 32}' '{"loads_per_lane": 48}' '{"loads_per_lane": 72}' '{"loads_per_lane": 74}'; do
    timeout -k 10 200 python3 bench.py --workload cfg4 --no-cpu --tune "$t" > gpurun_out/pb4_one.json 2>> gpurun_out/pb4_ab.err || exit 1
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/pb4_one.json').read().strip().splitlines()[-1]); r=d['roofline']
print(json.dumps({'what': 'cfg4', 'round': $r, 'tune': $t, 'kernel': r['kernel'].split('(')[0], 'kernel_ms': r['kernel_ms'], 'frac': r['frac']}))" >> gpurun_out/pb4_ab.jsonl
  done
done
for t in '{}' '{"loads_per_lane": 32}' '{"loads_per_lane": 28}'; do
  timeout -k 10 300 python3 tools/rx_device_bench.py --rings none --tune "$t" >> gpurun_out/pb4_ab.jsonl 2>> gpurun_out/pb4_ab.err || exit 1
done
cat gpurun_out/pb4_ab.jsonl

#!/bin/bash
# Round 6: ring parity tests, then the bench rings (tools/rx_device_bench.py)
# under the schedules named in $ARMS, one box.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_rx.py tests/test_gpu_bounds.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "ring" > gpurun_out/pytest_ring.log 2>&1 || { tail -40 gpurun_out/pytest_ring.log; exit 1; }
  tail -1 gpurun_out/pytest_ring.log
fi
timeout -k 10 500 python3 -u tools/rx_device_bench.py --skip-packed ${RINGS:+--rings $RINGS} ${ARMS:+--arms $ARMS} \
  ${TUNES:+--tunes "$(cat $TUNES)"} \
  > gpurun_out/${TAG:-r06_ring}.jsonl 2> gpurun_out/${TAG:-r06_ring}.err || { tail -20 gpurun_out/${TAG:-r06_ring}.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/${TAG:-r06_ring}.jsonl'):
    d = json.loads(l); print(d['what'], d['schedule'], d['ms'], d['frac'], d['last_kernel'][-20:])"

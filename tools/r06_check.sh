#!/bin/bash
# Round-6 check on the GPU box: the whole -m gpu suite, then short bench lines
# for the workloads named in $BENCH (default cfg5 cfg2), each step under its own
# time limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 420 python3 -u -m pytest tests -m gpu ${PYTEST_X:--x} -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} \
    > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
for c in ${BENCH:-cfg5 cfg2}; do
  timeout -k 10 300 python3 bench.py --workload $c --no-cpu > gpurun_out/b6_$c.json 2> gpurun_out/b6_$c.err \
    || { tail -5 gpurun_out/b6_$c.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/b6_$c.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$c', d['value'], d['ms_per_step'], r.get('kernel_ms'), r['frac'], r.get('kernel'))"
done

set -u
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 600 python3 -u -m pytest tests/test_multirank_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_mr.log 2>&1 || { tail -30 gpurun_out/pytest_mr.log; exit 1; }
tail -1 gpurun_out/pytest_mr.log
for c in cfg1 cfg4 cfg5; do
  timeout -k 10 300 python3 bench.py --workload $c --no-cpu > gpurun_out/bq_$c.json 2> gpurun_out/bq_$c.err || { tail -5 gpurun_out/bq_$c.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/bq_$c.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$c', d['value'], d['ms_per_step'], r['kernel_ms'], r['kernel_ms_b2b_mean'], r['frac'], r.get('frac_rocprof'), r['traffic_source'])"
done

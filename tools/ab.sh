#!/usr/bin/env bash
# GPU box: parity tests, then an A/B (each build in its own process) of the current build against
# the libraries named in $AB (default pip_amd/lib/ab/*.so).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG="${TAG:-ab}"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu.log
fi
timeout -k 10 900 python3 -u tools/ab_scan.py ${ONLY:+--only $ONLY} ${ROUNDS:+--rounds $ROUNDS} ${WARM:+--warm $WARM} ${B2B:+--b2b} ${AB:-pip_amd/lib/ab/*.so} \
  > "gpurun_out/$TAG.jsonl" 2> "gpurun_out/$TAG.err" || { echo "ab rc=$?"; tail -20 "gpurun_out/$TAG.err"; exit 1; }
cat "gpurun_out/$TAG.jsonl"

#!/usr/bin/env bash
# k_hdr A/B on one box: GPU tests (TESTS_K filter, all GPU tests by default), then
# cfg1 size scan over tools/arms_hdr.json (SIZES in Mi headers).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${TESTS_K:+-k "$TESTS_K"} \
  > gpurun_out/hdr_tests.log 2>&1; rc=$?
tail -8 gpurun_out/hdr_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 600 python3 tools/size_scan.py --only cfg1 --sizes "${SIZES:-1,16,64,256}" --arms @tools/arms_hdr.json \
  > gpurun_out/hdr_ab.jsonl 2> gpurun_out/hdr_ab.err || { echo "ab rc=$?"; tail -20 gpurun_out/hdr_ab.err; exit 1; }
cat gpurun_out/hdr_ab.jsonl

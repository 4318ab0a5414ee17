# k_flat_coop rows on the absolute 1 KiB grid: the parity tests, then the bench line against the build before (pip_amd/lib/ab/libpipck_base.so) on cfg5 / cfg3 / cfg2
set -u
cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_align.log 2>&1 || { tail -30 gpurun_out/pytest_align.log; exit 1; }
tail -1 gpurun_out/pytest_align.log
for c in cfg5 cfg3 cfg2; do
  ARMS="base=pip_amd/lib/ab/libpipck_base.so cur=pip_amd/lib/libpipck.so" ROUNDS=2 WL=$c TAG=align_$c bash tools/bench_ab.sh > /dev/null || exit 1
  cat gpurun_out/align_$c.jsonl
done

set -u
mkdir -p gpurun_out/scan
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "known_answer or thread_safe or zero_copy" > gpurun_out/pytest_res.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_res.log; exit 1; }
tail -1 gpurun_out/pytest_res.log
timeout -k 10 300 pip_amd/lib/percall_bench 2000 > gpurun_out/scan/percall.jsonl 2> gpurun_out/scan/percall.err || { echo "percall rc=$?"; tail gpurun_out/scan/percall.err; exit 1; }

set -u
mkdir -p gpurun_out/scan
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 900 python3 -u tools/ab_scan.py --only cfg2,cfg3,cfg4,cfg5,cfg4d pip_amd/lib/ab/libpipck_base.so > gpurun_out/scan/ab_buf.jsonl 2> gpurun_out/scan/ab_buf.err || exit 1

set -u
mkdir -p gpurun_out/scan
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "known_answer or thread_safe" > gpurun_out/pytest_res.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_res.log; exit 1; }
tail -1 gpurun_out/pytest_res.log
PIPCK_RESIDENT_VRAM=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "resident" > gpurun_out/pytest_res2.log 2>&1 || { echo "pytest vram failed"; tail -30 gpurun_out/pytest_res2.log; exit 1; }
tail -1 gpurun_out/pytest_res2.log
timeout -k 10 300 pip_amd/lib/percall_bench 2000 > gpurun_out/scan/percall.jsonl 2> gpurun_out/scan/percall.err || { echo "percall rc=$?"; tail gpurun_out/scan/percall.err; exit 1; }
PIPCK_RESIDENT_VRAM=1 timeout -k 10 300 pip_amd/lib/percall_bench 2000 > gpurun_out/scan/percall_vram.jsonl 2> gpurun_out/scan/percall_vram.err || { echo "percall vram rc=$?"; tail gpurun_out/scan/percall_vram.err; exit 1; }

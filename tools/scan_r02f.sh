set -u
mkdir -p gpurun_out/scan
timeout -k 10 60 oracle/_ref/stack_tx_amd --mode capture --bytes 1000000 > gpurun_out/scan/cold.json 2>&1 && timeout -k 10 60 oracle/_ref/stack_tx_amd --mode sync --bytes 100000 >> gpurun_out/scan/cold.json 2>&1 || exit 1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 600 python3 -u tools/ab_scan.py --only cfg2,cfg3,cfg4,cfg5 pip_amd/lib/ab/libpipck_base.so > gpurun_out/scan/ab_reorder.jsonl 2> gpurun_out/scan/ab_reorder.err || exit 1
timeout -k 10 300 python3 tools/size_scan.py --only cfg2,cfg3 --arms '{"default": {}, "queue": {"flat_queue": true}}' > gpurun_out/scan/queue2.jsonl 2> gpurun_out/scan/queue2.err

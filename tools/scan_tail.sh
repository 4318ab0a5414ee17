set -u
mkdir -p gpurun_out/scan
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "tail_queue or flat_stream" > gpurun_out/pytest_tail.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_tail.log; exit 1; }
tail -1 gpurun_out/pytest_tail.log
timeout -k 10 400 python3 tools/size_scan.py --only cfg2,cfg3 --arms '{"default": {}, "tail": {"flat_tail_queue": true}}' > gpurun_out/scan/tail.jsonl 2> gpurun_out/scan/tail.err || exit 1
timeout -k 10 300 python3 tools/size_scan.py --only cfg5 --sizes 8 --arms '{"default": {}, "tail": {"flat_tail_queue": true}}' >> gpurun_out/scan/tail.jsonl 2>> gpurun_out/scan/tail.err || exit 1
timeout -k 10 400 python3 tools/task_trace.py --only cfg2 --arms '{"default": {}, "tail": {"flat_tail_queue": true}}' --dump gpurun_out/trace/npy5 > gpurun_out/trace/trace5.jsonl 2> gpurun_out/trace/trace5.err

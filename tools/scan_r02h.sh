set -u
mkdir -p gpurun_out/scan gpurun_out/trace
timeout -k 10 300 python3 tools/size_scan.py --only cfg2,cfg3 --arms '{"default": {}, "queue": {"flat_queue": true}}' > gpurun_out/scan/queue3.jsonl 2> gpurun_out/scan/queue3.err || exit 1
timeout -k 10 300 python3 tools/size_scan.py --only cfg5 --sizes 8 --arms '{"default": {}, "queue": {"flat_queue": true}}' >> gpurun_out/scan/queue3.jsonl 2>> gpurun_out/scan/queue3.err || exit 1
timeout -k 10 400 python3 tools/task_trace.py --only cfg2,cfg3 --arms '{"default": {}, "queue": {"flat_queue": true}}' --dump gpurun_out/trace/npy3 > gpurun_out/trace/trace3.jsonl 2> gpurun_out/trace/trace3.err

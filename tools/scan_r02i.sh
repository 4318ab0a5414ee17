set -u
mkdir -p gpurun_out/scan gpurun_out/trace
timeout -k 10 300 python3 tools/size_scan.py --only cfg2,cfg3 --arms '{"default": {}, "cont": {"flat_queue": true}}' > gpurun_out/scan/cont.jsonl 2> gpurun_out/scan/cont.err || exit 1
timeout -k 10 300 python3 tools/size_scan.py --only cfg5 --sizes 8 --arms '{"default": {}, "cont": {"flat_queue": true}}' >> gpurun_out/scan/cont.jsonl 2>> gpurun_out/scan/cont.err || exit 1
timeout -k 10 400 python3 tools/task_trace.py --only cfg2,cfg3 --arms '{"default": {}, "cont": {"flat_queue": true}}' --dump gpurun_out/trace/npy4 > gpurun_out/trace/trace4.jsonl 2> gpurun_out/trace/trace4.err

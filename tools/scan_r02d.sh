set -u
mkdir -p gpurun_out/trace gpurun_out/scan
timeout -k 10 400 python3 tools/task_trace.py --only cfg2,cfg5,cfg3 --arms '{"default": {}, "one_wave": {"flat_one_wave": true}}' > gpurun_out/trace/trace_onewave.jsonl 2> gpurun_out/trace/trace.err || exit 1
timeout -k 10 400 python3 tools/size_scan.py --only cfg2,cfg3,cfg5 --sizes 4 --arms '{"default": {}, "one_wave": {"flat_one_wave": true}}' > gpurun_out/scan/onewave.jsonl 2> gpurun_out/scan/onewave.err

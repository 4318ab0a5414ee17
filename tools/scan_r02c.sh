set -u
mkdir -p gpurun_out/trace
timeout -k 10 400 python3 tools/task_trace.py --only cfg2,cfg4,cfg5,cfg3 --dump gpurun_out/trace/npy > gpurun_out/trace/trace.jsonl 2> gpurun_out/trace/trace.err

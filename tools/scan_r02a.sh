set -u
mkdir -p gpurun_out/scan
mkdir -p gpurun_out/stack_tx; rm -f gpurun_out/stack_tx/*
timeout -k 10 600 bash tools/stack_tx.sh > gpurun_out/stack_tx/log.txt 2>&1 || exit 1
timeout -k 10 300 python3 tools/size_scan.py --only cfg4 --packed --sizes 8 --arms '{"default": {}, "plain": {"plain_loads": true}, "ring16": {"loads_per_lane": 17}, "ring32": {"loads_per_lane": 33}, "marks": {"packed_marks_only": true}}' > gpurun_out/scan/cfg4.jsonl 2> gpurun_out/scan/cfg4.err || exit 1
timeout -k 10 300 python3 tools/size_scan.py --only cfg2 --arms '{"default": {}, "rows128": {"rows_per_task": 128}, "rows96": {"rows_per_task": 96}, "r16_rows128": {"loads_per_lane": 17, "rows_per_task": 128}, "ring32": {"loads_per_lane": 33}, "plain": {"plain_loads": true}, "ring16": {"loads_per_lane": 17}}' > gpurun_out/scan/cfg2.jsonl 2> gpurun_out/scan/cfg2.err

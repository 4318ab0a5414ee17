set -u
mkdir -p gpurun_out/scan
timeout -k 10 300 python3 tools/size_scan.py --only cfg2,cfg3 --arms '{"default": {}, "cont": {"flat_queue": true}, "cont_static": {"flat_queue": true, "cont_static": true}, "cont_r16": {"flat_queue": true, "loads_per_lane": 17}}' > gpurun_out/scan/cont2.jsonl 2> gpurun_out/scan/cont2.err

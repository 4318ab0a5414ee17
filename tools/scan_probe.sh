set -u
mkdir -p gpurun_out/scan
timeout -k 10 400 python3 tools/size_scan.py --only cfg2,cfg3 --arms '{"default": {}, "loads_probe": {"loads_only": true}}' > gpurun_out/scan/probe.jsonl 2> gpurun_out/scan/probe.err || exit 1
timeout -k 10 300 python3 tools/size_scan.py --only cfg5 --sizes 8 --arms '{"default": {}, "loads_probe": {"loads_only": true}}' >> gpurun_out/scan/probe.jsonl 2>> gpurun_out/scan/probe.err

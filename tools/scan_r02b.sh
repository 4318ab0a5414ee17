set -u
mkdir -p gpurun_out/scan
timeout -k 10 300 python3 tools/size_scan.py --only cfg2 --sizes 1,2,4,8,16,32 --arms '{"default": {}}' > gpurun_out/scan/cfg2_sizes.jsonl 2> gpurun_out/scan/cfg2_sizes.err || exit 1
timeout -k 10 300 python3 tools/size_scan.py --only cfg4 --packed --sizes 2,4,8,16,32 --arms '{"default": {}}' > gpurun_out/scan/cfg4_sizes.jsonl 2> gpurun_out/scan/cfg4_sizes.err || exit 1
timeout -k 10 300 python3 tools/size_scan.py --only cfg5 --sizes 0.25,0.5,1,2,8 --arms '{"default": {}}' > gpurun_out/scan/cfg5_sizes.jsonl 2> gpurun_out/scan/cfg5_sizes.err

set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
A='{"default": {}}'
timeout -k 10 300 python3 tools/size_scan.py --only cfg2 --sizes 1,2,4,8,16,32 --arms "$A" > gpurun_out/size_r03.jsonl 2> gpurun_out/size_r03.err || exit 1
timeout -k 10 300 python3 tools/size_scan.py --only cfg4 --packedb --sizes 2,4,8,16,32 --arms "$A" >> gpurun_out/size_r03.jsonl 2>> gpurun_out/size_r03.err || exit 1
timeout -k 10 300 python3 tools/size_scan.py --only cfg5 --sizes 1,2,4,8,16 --arms "$A" >> gpurun_out/size_r03.jsonl 2>> gpurun_out/size_r03.err || exit 1
timeout -k 10 300 python3 tools/size_scan.py --only cfg3 --sizes 1,4,8 --arms "$A" >> gpurun_out/size_r03.jsonl 2>> gpurun_out/size_r03.err || exit 1
timeout -k 10 300 python3 tools/size_scan.py --only cfg1 --sizes 8,32,128,256,512 --arms "$A" >> gpurun_out/size_r03.jsonl 2>> gpurun_out/size_r03.err || exit 1
cat gpurun_out/size_r03.jsonl | cut -c1-200

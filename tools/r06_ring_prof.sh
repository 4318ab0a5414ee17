#!/bin/bash
# rocprofv3 kernel trace of the ring bench (default arm) on the rings in $RINGS:
# per-kernel durations.
set -u
R="${GRAFT_REPO_ROOT:-$PWD}"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG:-ringprof}" -o ring --output-format csv -- \
  python3 "$R/tools/rx_device_bench.py" --skip-packed --rings "${RINGS:-ring_dense_9216,ring_sparse_9216}" \
  --arms "${ARMS:-groups}" --rounds 1 --warm 5 --iters 5 > "$R/gpurun_out/${TAG:-ringprof}.out" 2>&1 || { tail -20 "$R/gpurun_out/${TAG:-ringprof}.out"; exit 1; }
cat "$R/gpurun_out/${TAG:-ringprof}.out" | grep what
f=$(find "$R/gpurun_out/${TAG:-ringprof}" -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 "$f" | head -12
k=$(find "$R/gpurun_out/${TAG:-ringprof}" -name "*kernel_trace.csv" | head -1)
python3 - "$k" <<PY
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if "k_ring" in r["Kernel_Name"]:
        print(r["Kernel_Name"][:40], int(r["Start_Timestamp"]) % 10**10, int(r["End_Timestamp"]) % 10**10, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
PY

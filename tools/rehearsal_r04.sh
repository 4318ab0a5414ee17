#!/usr/bin/env bash
# N-rank rehearsal lines on one GPU (ranks share it: --share-gpus), round 4:
# the SURVEY 8e aggregate (latest end - earliest start) and its timing fields.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/rehearsal_r04
mkdir -p "$OUT"
run() {  # $1 = name, rest = command
  local name=$1; shift
  timeout -k 10 300 "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "$name rc=$?"; tail -5 "$OUT/$name.err"; exit 1; }
  grep '^{' "$OUT/$name.json" | tail -1
}
run n2_self python3 bench.py --gpus 2 --share-gpus --packets-per-gpu 2097152 --no-cpu
run n4_self python3 bench.py --gpus 4 --share-gpus --packets-per-gpu 1048576 --no-cpu
run n2_torchrun python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --share-gpus --packets-per-gpu 2097152 --no-cpu
run n2_skew50 python3 bench.py --gpus 2 --share-gpus --packets-per-gpu 2097152 --no-cpu --start-skew-ms 50
echo "== rehearsal done"

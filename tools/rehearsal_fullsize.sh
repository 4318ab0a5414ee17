# N = 2 at the headline's full per-GPU size (cfg5, 8M x 8,980 B = 75 GB per
# rank), both ranks sharing the box's one GPU (150 GB of its 288 GB), launched
# as the driver launches N > 1: torch.distributed.run, one line from rank 0.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --share-gpus --steps 10 --warmup 20 --no-cpu \
  > gpurun_out/rehearsal_2rank_fullsize.json 2> gpurun_out/rehearsal_2rank_fullsize.err || { echo "rc=$?"; tail -20 gpurun_out/rehearsal_2rank_fullsize.err; exit 1; }
tail -1 gpurun_out/rehearsal_2rank_fullsize.json | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print(json.dumps({k: d[k] for k in ('value','n_gpus','ms_per_step','distinct_gpus')} | {'per_rank_gib_per_s': d['per_rank_gib_per_s'], 'kernel_ms': r['kernel_ms'], 'frac': r['frac'], 'parallelism': d['config']['parallelism'], 'global_packets': d['config']['global_packets'], 'timing': d['timing']}))"

"""GPU, N>1: two processes (sharing the box's GPU when only one is visible).

* each rank generates and checksums its own contiguous shard in its own HBM
  arena; the concatenated results equal a single-process run (no data-path
  collective -- gloo only carries the comparison back);
* bench.py under torch.distributed.run prints one JSON line with n_gpus = 2,
  weak scaling and the whole-job packet count.
"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, n_total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch

    from pip_amd import engine, shard
    from pip_amd.workloads import CFG2, N_FLOWS

    env = shard.dist_env()
    shard.init_control_plane(env)
    torch.cuda.set_device(env.local_rank % torch.cuda.device_count())
    w = CFG2
    first, count = shard.shard_range(n_total, env.world, env.rank)
    arena = torch.empty(count * w.stride, dtype=torch.uint8, device="cuda")
    engine.gen_fixed(arena, w.stride, w.length, count, first, w.seed, w.hdr)
    _, pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)
    out = engine.checksum_fixed(arena, w.stride, w.length, count, pseudo, N_FLOWS, None, first)
    q.put((rank, out.cpu().numpy().view(np.uint16).tobytes()))
    shard.barrier(env)
    shard.shutdown(env)


def test_two_ranks_equal_one(oracle):
    import torch
    import torch.multiprocessing as mp

    n_total = 50_001
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_rank, args=(r, 2, port, n_total, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    got = np.frombuffer(b"".join(r[1] for r in res), dtype=np.uint16)
    from pip_amd import engine
    from pip_amd.workloads import CFG2, N_FLOWS

    w = CFG2
    arena = torch.empty(n_total * w.stride, dtype=torch.uint8, device="cuda")
    engine.gen_fixed(arena, w.stride, w.length, n_total, 0, w.seed, w.hdr)
    _, pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)
    one = engine.checksum_fixed(arena, w.stride, w.length, n_total, pseudo, N_FLOWS).cpu().numpy().view(np.uint16)
    assert np.array_equal(got, one)
    host = oracle.gen_fixed_batch(w.seed, 0, 2000, w.length, w.hdr, w.stride)
    assert np.array_equal(one[:2000], oracle.batch_fixed(host, w.stride, w.length, 2000, 4, 6, w.seed, N_FLOWS, 0))


def test_bench_two_ranks_json_contract():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "bench.py"), "--gpus", "2",
           "--steps", "3", "--warmup", "1", "--packets-per-gpu", "200000"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["steps"] == 3
    assert d["config"]["global_packets"] == 400000 and d["config"]["packets_per_gpu"] == 200000
    assert d["value"] > 0 and d["roofline"]["bound"] == "hbm" and d["cpu_baseline"] is None

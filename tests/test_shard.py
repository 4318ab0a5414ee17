"""CPU: the N>1 path.  Shards are contiguous global packet-id ranges; each rank
checksums its own shard with no data-path collective; the union over ranks is
byte- and result-identical to a single-rank run.  world_size 2 over gloo."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from pip_amd import shard
from pip_amd.workloads import CFG2, CFG4, N_FLOWS


def test_shard_range_partitions_exactly():
    for n in (0, 1, 7, 1000, 64 << 20):
        for world in (1, 2, 3, 4, 8):
            parts = [shard.shard_range(n, world, r) for r in range(world)]
            assert parts[0][0] == 0
            assert sum(c for _, c in parts) == n
            for (f0, c0), (f1, _) in zip(parts, parts[1:]):
                assert f0 + c0 == f1
            assert max(c for _, c in parts) - min(c for _, c in parts) <= 1


def test_shard_by_bytes_balances_ragged():
    rng = np.random.default_rng(3)
    lens = rng.integers(64, 9000, 5000)
    prefix = [0] + list(np.cumsum(lens))
    for world in (1, 2, 4, 8):
        parts = [shard.shard_by_bytes(prefix, world, r) for r in range(world)]
        assert sum(c for _, c in parts) == len(lens)
        per = [prefix[f + c] - prefix[f] for f, c in parts]
        assert max(per) - min(per) <= 2 * 9000


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from oracle.oracle import Oracle

    env = shard.dist_env()
    shard.init_control_plane(env)
    orc = Oracle()
    n_total = 3000
    w = CFG2
    first, count = shard.shard_range(n_total, env.world, env.rank)
    arena = orc.gen_fixed_batch(w.seed, first, count, w.length, w.hdr, w.stride)
    out = orc.batch_fixed(arena, w.stride, w.length, count, w.family, w.proto, w.seed, N_FLOWS, first)
    shard.barrier(env)
    t = shard.max_over_ranks(env, float(rank + 1))
    total = shard.sum_over_ranks(env, float(count))
    q.put((rank, first, out.tobytes(), t, total))
    shard.shutdown(env)


def test_gloo_world2_shards_equal_single_run(oracle):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    w = CFG2
    arena = oracle.gen_fixed_batch(w.seed, 0, 3000, w.length, w.hdr, w.stride)
    single = oracle.batch_fixed(arena, w.stride, w.length, 3000, w.family, w.proto, w.seed, N_FLOWS, 0)
    joined = np.frombuffer(b"".join(r[2] for r in res), dtype=np.uint16)
    assert np.array_equal(joined, single)
    assert all(r[3] == 2.0 for r in res)      # MAX over ranks
    assert all(r[4] == 3000.0 for r in res)   # units all ranks processed


@pytest.mark.parametrize("world", [2, 4, 8])
def test_ragged_shards_regenerate_identically(oracle, world):
    """cfg4: a rank regenerates packets from global ids, so its bytes do not
    depend on the GPU count."""
    w = CFG4
    n = 400
    whole, offs, lens = oracle.gen_ragged_batch(w.seed, 0, n, w.hdr)
    for r in range(world):
        first, count = shard.shard_range(n, world, r)
        part, poffs, plens = oracle.gen_ragged_batch(w.seed, first, count, w.hdr)
        assert np.array_equal(plens, lens[first:first + count])
        for i in range(count):
            a = whole[int(offs[first + i]):int(offs[first + i]) + int(lens[first + i])]
            b = part[int(poffs[i]):int(poffs[i]) + int(plens[i])]
            assert np.array_equal(a, b)


def test_byte_cuts_match_shard_by_bytes():
    import torch

    rng = np.random.default_rng(11)
    lens = rng.integers(64, 9001, 20000)
    prefix = [0] + [int(x) for x in np.cumsum(lens)]
    for world in (1, 2, 3, 4, 8):
        want = [shard.shard_by_bytes(prefix, world, r) for r in range(world)]
        for arr in (np.array(prefix, dtype=np.int64), torch.tensor(prefix, dtype=torch.int64)):
            cuts = shard.byte_cuts(arr, world)
            assert [(cuts[r], cuts[r + 1] - cuts[r]) for r in range(world)] == want


_RANK_SCRIPT = """
import os, sys
sys.path.insert(0, {root!r})
from pip_amd import shard
env = shard.dist_env()
shard.init_control_plane(env)
got = shard.gather_over_ranks(env, [float(env.rank), float(env.local_rank), float(env.world)])
shard.barrier(env)
if env.rank == 0:
    print("RANKS", got, flush=True)
if env.rank == {fail_rank}:
    sys.exit(7)
shard.shutdown(env)
"""


@pytest.mark.parametrize("fail_rank", [-1, 1])
def test_spawn_ranks_runs_a_gloo_job(tmp_path, capfd, fail_rank):
    """bench.py's self-launch: N children with RANK/LOCAL_RANK/WORLD_SIZE and a
    rendezvous on 127.0.0.1; a failing rank's status comes back."""
    from pathlib import Path
    import sys

    root = str(Path(__file__).resolve().parents[1])
    script = tmp_path / "rank.py"
    script.write_text(_RANK_SCRIPT.format(root=root, fail_rank=fail_rank))
    rc = shard.spawn_ranks(3, [sys.executable, str(script)])
    out = capfd.readouterr().out
    assert "RANKS [[0.0, 0.0, 3.0], [1.0, 1.0, 3.0], [2.0, 2.0, 3.0]]" in out
    assert rc == (7 if fail_rank == 1 else 0)


def test_bench_refuses_world_size_mismatch(monkeypatch):
    """Under torch.distributed.run, WORLD_SIZE must equal --gpus (checked before
    anything touches the GPU)."""
    import bench

    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.main(["--gpus", "4"]) == 2
    monkeypatch.setenv("WORLD_SIZE", "1")
    assert bench.main(["--gpus", "2"]) == 2


def test_workload_text_states_the_real_count():
    from pip_amd.workloads import CFG1, CFG5

    assert CFG5.describe(64 << 20, 8).endswith("64M packets over 8 GPUs")
    assert CFG1.describe(256 << 20) .endswith("256M packets")
    assert CFG1.describe(1000).endswith("1,000 packets")
    assert CFG1.stride == 20 == CFG1.length  # packed headers: no slot padding


_N8_SCRIPT = """
import json, socket, sys, time
sys.path.insert(0, {root!r})
from pip_amd import shard
env = shard.dist_env()
shard.init_control_plane(env)
# bench.py's run_rank on an 8-GPU node, minus the GPU: device choice, timed
# region, the gathers and the aggregate, in bench.py's order
dev = shard.device_for_rank(env.local_rank, shard.local_world_size(env), 8, False)
place = {{"rank": env.rank, "host": socket.gethostname(), "device": dev, "pci_bus_id": "0000:%02x:00.0" % (16 * dev)}}
t0, t1 = shard.timed_steps(env, 5, lambda i: time.sleep(0.01), lambda: None)
ranks = shard.gather_over_ranks(env, [1e9, 1000.0, (t1 - t0) / 1e9, 0.002])
clocks = shard.gather_ints(env, [t0, t1])
places = shard.gather_objects(env, place)
agg = shard.aggregate([c[0] for c in clocks], [c[1] for c in clocks], [r[0] for r in ranks], 5)
shard.barrier(env)
if env.rank == 0:
    print("N8 " + json.dumps({{"world": env.world, "local_world": shard.local_world_size(env), "agg": agg,
                              "devices": [p["device"] for p in places],
                              "distinct": len({{(p["host"], p["pci_bus_id"]) for p in places}})}}), flush=True)
shard.shutdown(env)
"""


@pytest.mark.parametrize("launcher", ["spawn", "torchrun"])
def test_eight_rank_control_plane_rehearsal(tmp_path, capfd, launcher):
    """The N=8 SCALE line's control plane on CPU (gloo, 8 processes): each local
    rank takes its own device of an 8-GPU node, the gathers return all eight
    ranks, and the aggregate is 8 shards' bytes over the shared-clock span --
    self-launched (bench.py --gpus 8) and under torch.distributed.run as the
    driver launches it."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    root = str(Path(__file__).resolve().parents[1])
    script = tmp_path / "n8.py"
    script.write_text(_N8_SCRIPT.format(root=root))
    if launcher == "spawn":
        assert shard.spawn_ranks(8, [sys.executable, str(script)]) == 0
        out = capfd.readouterr().out
    else:
        r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                            "--master-addr", "127.0.0.1", "--master-port", str(shard.free_port()), str(script)],
                           capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        out = r.stdout
    got = json.loads(next(ln for ln in out.splitlines() if ln.startswith("N8 "))[3:])
    assert got["world"] == 8 and got["local_world"] == 8
    assert got["devices"] == list(range(8)) and got["distinct"] == 8
    agg = got["agg"]
    assert agg["span_s"] >= agg["max_rank_s"] > 0.04
    assert agg["rate"] == pytest.approx(8 * 1e9 * 5 / agg["span_s"])

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


def n_visible() -> int:
    import torch

    return torch.cuda.device_count()


def share_flag(world: int) -> list[str]:
    """--share-gpus only where the box has fewer GPUs than ranks (bench.py refuses otherwise)."""
    return ["--share-gpus"] if world > n_visible() else []


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


def _ragged_rank(rank, world, port, n_total, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch

    from pip_amd import engine, shard
    from pip_amd.workloads import CFG4, N_FLOWS

    env = shard.dist_env()
    shard.init_control_plane(env)
    torch.cuda.set_device(env.local_rank % torch.cuda.device_count())
    w = CFG4
    lens_all = torch.empty(n_total, dtype=torch.int32, device="cuda")
    engine.call("pipck_gen_zipf_lengths", engine._ptr(lens_all), n_total, 0, w.seed, engine.current_stream())
    prefix = torch.zeros(n_total + 1, dtype=torch.int64, device="cuda")
    torch.cumsum(lens_all.to(torch.int64), 0, out=prefix[1:])
    cuts = shard.byte_cuts(prefix, world)
    first, count = cuts[rank], cuts[rank + 1] - cuts[rank]
    arena, desc, lens = engine.gen_ragged(count, first, w.seed, w.hdr, N_FLOWS,
                                          lengths=lens_all[first:first + count].clone())
    _, pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)
    out = engine.checksum_ragged(arena, desc, pseudo)
    q.put((rank, int(lens.to(torch.int64).sum().item()), out.cpu().numpy().view(np.uint16).tobytes()))
    shard.barrier(env)
    shard.shutdown(env)


def test_two_ranks_ragged_equal_bytes(oracle):
    """cfg4 split at equal L4 bytes (shard.byte_cuts): the two shards' results
    concatenate to the one-rank answer, and the byte split is balanced."""
    import torch
    import torch.multiprocessing as mp

    from pip_amd import engine
    from pip_amd.workloads import CFG4, N_FLOWS

    n_total = 60_007
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_ragged_rank, args=(r, 2, port, n_total, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    b0, b1 = res[0][1], res[1][1]
    assert abs(b0 - b1) <= 2 * 9000, (b0, b1)  # cut at a packet boundary: within one packet of half
    got = np.frombuffer(b"".join(r[2] for r in res), dtype=np.uint16)
    w = CFG4
    arena, desc, _ = engine.gen_ragged(n_total, 0, w.seed, w.hdr, N_FLOWS)
    _, pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)
    one = engine.checksum_ragged(arena, desc, pseudo).cpu().numpy().view(np.uint16)
    assert np.array_equal(got, one)
    h_arena, offs, lens = oracle.gen_ragged_batch(w.seed, 0, 3000, w.hdr)
    assert np.array_equal(one[:3000], oracle.batch_ragged(h_arena, offs, lens, 4, 6, w.seed, N_FLOWS, 0))


def test_bench_self_launch_cfg5_two_ranks():
    """`python bench.py --gpus 2` with no torchrun: bench.py starts both ranks
    itself (sharing the box's one GPU), each with a full cfg5 shard of 8M
    8,980-byte packets (2 x 75 GB of HBM), and rank 0 prints one JSON line."""
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1", "--no-cpu",
           *share_flag(2)]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert d["config"]["global_packets"] == 2 * (8 << 20) and d["config"]["packets_per_gpu"] == 8 << 20
    assert d["config"]["workload"].startswith("cfg5_tcp4_mtu9000") and "16M packets over 2 GPUs" in d["config"]["workload"]
    assert len(d["per_rank_gib_per_s"]) == 2 and all(v > 0 for v in d["per_rank_gib_per_s"])
    assert d["per_rank_packets"] == [8 << 20, 8 << 20]


def test_bench_two_ranks_json_contract():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "bench.py"), "--gpus", "2",
           "--steps", "3", "--warmup", "1", "--packets-per-gpu", "200000", *share_flag(2)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak" and d["steps"] == 3
    assert d["config"]["global_packets"] == 400000 and d["config"]["packets_per_gpu"] == 200000
    assert d["value"] > 0 and d["roofline"]["bound"] == "hbm" and d["cpu_baseline"] is None
    assert len(d["per_rank_gib_per_s"]) == 2
    # value over the span from the earliest start to the latest end
    t = d["timing"]
    assert t["value_over"].startswith("latest end - earliest start")
    assert t["span_ms"] >= t["max_rank_elapsed_ms"] and t["start_skew_ms"] >= 0
    assert d["value"] <= t["value_by_max_rank_elapsed"] + 0.01
    assert d["ms_per_step"] == pytest.approx(t["span_ms"] / 3, rel=1e-3)


def test_bench_start_skew_lowers_the_value():
    """An injected start skew after the barrier (rank 1 starts 200 ms late) shows
    in the line: start_skew_ms, and a value below the max-rank-elapsed figure."""
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--packets-per-gpu", "200000", "--no-cpu", "--start-skew-ms", "200", *share_flag(2)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=_bench_env())
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    t = d["timing"]
    assert 190 < t["start_skew_ms"] < 400 and t["injected_start_skew_ms_per_rank"] == 200
    assert t["span_ms"] >= t["max_rank_elapsed_ms"] + 190
    assert d["value"] < 0.5 * t["value_by_max_rank_elapsed"]


def test_bench_cfg4_two_ranks_byte_split():
    """The ragged bench under two ranks splits the global Zipf batch at equal bytes."""
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--workload", "cfg4", "--steps", "2",
           "--warmup", "1", "--packets-per-gpu", "300000", "--no-cpu", *share_flag(2)]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert d["config"]["global_packets"] == 600000 and sum(d["per_rank_packets"]) == 600000
    assert "equal bytes" in d["config"]["parallelism"]


def _bench_env():
    return {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}


def test_bench_four_ranks_share_flag_and_placement():
    """an N-rank line cannot claim more GPUs than it ran on.
    On a box with fewer than 4 GPUs, `bench.py --gpus 4` without --share-gpus
    exits non-zero before any timed work; with the flag it runs 4 ranks, prints
    four per-rank device records (device index + PCI bus id), says the GPUs were
    shared, and the global packet count is the sum of the shards."""
    if n_visible() >= 4:
        pytest.skip("4+ GPUs visible: sharing is not needed")
    base = [sys.executable, str(ROOT / "bench.py"), "--gpus", "4", "--steps", "2", "--warmup", "1",
            "--packets-per-gpu", "100000", "--no-cpu"]
    r = subprocess.run(base, capture_output=True, text=True, timeout=300, cwd=ROOT, env=_bench_env())
    assert r.returncode != 0
    assert "--share-gpus" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    r = subprocess.run(base + ["--share-gpus"], capture_output=True, text=True, timeout=600, cwd=ROOT,
                       env=_bench_env())
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 4 and d["distinct_gpus"] == n_visible()
    recs = d["per_rank_device"]
    assert [p["rank"] for p in recs] == [0, 1, 2, 3]
    assert all(p["pci_bus_id"] and p["device"] < n_visible() for p in recs)
    assert len({p["pci_bus_id"] for p in recs}) == n_visible()
    assert "SHARING" in d["config"]["parallelism"]
    assert d["per_rank_packets"] == [100000] * 4 and d["config"]["global_packets"] == sum(d["per_rank_packets"])


def test_bench_line_names_its_kernel_and_build():
    """The bench line names the kernel instantiation it timed (pipck_last_launch)
    and the libpipck.so build; traffic is attached only for that exact pair."""
    import hashlib

    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--workload", "cfg2", "--steps", "2", "--warmup", "1",
                        "--packets-per-gpu", "100000", "--no-cpu"], capture_output=True, text=True, timeout=300,
                       cwd=ROOT, env=_bench_env())
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    rf = d["roofline"]
    assert rf["kernel"].startswith("void pipck::k_flat_coop<32, false, true>(")
    from pip_amd import _lib

    assert rf["lib_sha256"] == hashlib.sha256(Path(_lib.LIBPIPCK).read_bytes()).hexdigest()
    # 100000 packets is not the profiled batch: no traffic may be attached
    assert rf["traffic"] is None and "mismatch" in rf["traffic_source"]
    assert d["per_rank_device"][0]["pci_bus_id"]


def test_bench_results_host_line():
    """`bench.py --results-host`: the kernel writes its results into pinned host
    memory; the line says so, attaches no PMC traffic (measured with HBM
    results), and the results still equal pip's own code on the host."""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--workload", "cfg2", "--steps", "2", "--warmup", "1",
                        "--packets-per-gpu", "65536", "--results-host"], capture_output=True, text=True, timeout=300,
                       cwd=ROOT, env=_bench_env())
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert d["config"]["results"].startswith("pinned host memory")
    assert d["roofline"]["traffic"] is None and "--results-host" in d["roofline"]["traffic_source"]
    assert d["cpu_baseline"]["gpu_results_match"] is True


@pytest.mark.parametrize("launcher", ["self", "torchrun"])
def test_bench_eight_ranks_rehearsal(launcher):
    """the driver's 8-GPU SCALE line, rehearsed on this box.
    `bench.py --gpus 8` self-launched and under torch.distributed.run
    --nproc-per-node 8, 1M cfg5 packets per rank: one JSON line with 8
    per_rank_device records, the distinct GPUs it really ran on (SHARING when the
    box has fewer than 8), and each rank's results digest -- rank 5's shard
    (packet ids 5M .. 6M) equals a one-rank run of the same ids here."""
    import hashlib

    import torch

    from pip_amd import engine
    from pip_amd.workloads import CFG5, N_FLOWS

    per = 1 << 20
    args = [str(ROOT / "bench.py"), "--gpus", "8", "--steps", "3", "--warmup", "1", "--packets-per-gpu", str(per),
            "--no-cpu", "--digest", *share_flag(8)]
    if launcher == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), *args]
    else:
        cmd = [sys.executable, *args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=ROOT, env=_bench_env())
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["scaling"] == "weak"
    assert d["config"]["global_packets"] == 8 * per and d["per_rank_packets"] == [per] * 8
    assert [p["rank"] for p in d["per_rank_device"]] == list(range(8))
    assert d["distinct_gpus"] == min(8, n_visible())
    if n_visible() < 8:
        assert f"8 ranks SHARING {n_visible()} GPU(s)" in d["config"]["parallelism"]
    recs = d["per_rank_results"]
    assert [(x["rank"], x["first"], x["count"]) for x in recs] == [(k, k * per, per) for k in range(8)]
    # a one-rank run of rank 5's packet ids, in this process
    w, first = CFG5, recs[5]["first"]
    arena = torch.empty(per * w.stride, dtype=torch.uint8, device="cuda")
    engine.gen_fixed(arena, w.stride, w.length, per, first, w.seed, w.hdr)
    _, pseudo = engine.gen_flows(w.family, N_FLOWS, w.seed, w.proto)
    one = engine.checksum_fixed(arena, w.stride, w.length, per, pseudo, N_FLOWS, None, first)
    assert hashlib.sha256(one.cpu().numpy().tobytes()).hexdigest() == recs[5]["sha256"]
    assert len({x["sha256"] for x in recs}) == 8  # every shard its own packets

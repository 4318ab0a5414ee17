"""Sharding of packet batches across GPUs.

Every packet is independent, so a batch is split into contiguous global
packet-id ranges, one per rank (one process per GPU).  There is no exchange
step and therefore no collective on the data path: each rank generates its
own shard on its own device from global packet ids and checksums it in
place.  The only cross-rank traffic is control: a barrier around the timed
region and every rank's start and end on the node's shared monotonic clock,
over gloo (CPU), so RCCL is never initialised.  The aggregate rate is
SURVEY.md 8e's: all ranks' units / (latest end - earliest start).
"""
from __future__ import annotations

import os
import time
from bisect import bisect_left
from dataclasses import dataclass


@dataclass(frozen=True)
class DistEnv:
    rank: int
    world: int
    local_rank: int

    @property
    def distributed(self) -> bool:
        return self.world > 1


def dist_env() -> DistEnv:
    """RANK / WORLD_SIZE / LOCAL_RANK as set by torch.distributed.run."""
    return DistEnv(int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
                   int(os.environ.get("LOCAL_RANK", 0)))


def free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(world: int, argv: list[str], port: int | None = None) -> int:
    """Run ``argv`` as ranks 0..world-1 of a one-node job (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT in each child's environment),
    the way ``torch.distributed.run --nnodes=1`` would.  The parent only waits:
    it never touches the GPU (the children each pick theirs by LOCAL_RANK).
    Returns 0, or the first failing rank's exit status (128 + signal for a
    signal) after terminating the ranks still running."""
    import subprocess
    import time

    port = port or free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(argv, env=env))
    rc, running = 0, set(range(world))
    while running:
        for r in sorted(running):
            code = procs[r].poll()
            if code is None:
                continue
            running.discard(r)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in running:
                    procs[q].terminate()
        time.sleep(0.02)
    return rc


def shard_range(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous, balanced packet-id range [first, first+count) of one rank."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    first = n_total * rank // world
    return first, n_total * (rank + 1) // world - first


def shard_by_bytes(prefix_bytes: list[int] | tuple[int, ...], world: int, rank: int) -> tuple[int, int]:
    """Ragged batches: split at packet boundaries so every rank gets ~equal bytes.

    ``prefix_bytes[i]`` is the byte offset where packet i starts; the last
    element is the total (len == n_packets + 1)."""
    n = len(prefix_bytes) - 1
    total = prefix_bytes[-1]

    def cut(r: int) -> int:
        if r <= 0:
            return 0
        if r >= world:
            return n
        return min(n, bisect_left(prefix_bytes, total * r // world))

    a, b = cut(rank), cut(rank + 1)
    return a, b - a


def byte_cuts(prefix_bytes, world: int) -> list[int]:
    """``shard_by_bytes`` for every rank at once over a large sorted prefix array
    (numpy array or torch tensor, len == n_packets + 1): the N+1 packet indices
    where the rank ranges begin/end.  ``searchsorted(side="left")`` is bisect_left."""
    n = len(prefix_bytes) - 1
    total = int(prefix_bytes[-1])
    cuts = [0]
    for r in range(1, world):
        target = total * r // world
        if hasattr(prefix_bytes, "cpu"):  # torch tensor (device-resident prefix)
            import torch

            at = int(torch.searchsorted(prefix_bytes, torch.tensor([target], dtype=prefix_bytes.dtype,
                                                                    device=prefix_bytes.device)).item())
        else:
            import numpy as np

            at = int(np.searchsorted(prefix_bytes, target, side="left"))
        cuts.append(min(n, at))
    cuts.append(n)
    return cuts


def device_for_rank(local_rank: int, local_world: int, n_devices: int, share: bool = False) -> int:
    """One GPU per rank: local rank r takes device r of its node.  More ranks on
    a node (``local_world``, torchrun's LOCAL_WORLD_SIZE) than GPUs visible there
    is refused unless ``share`` (a rehearsal of N>1 on fewer GPUs, which the
    bench line then reports as shared) -- so an N-GPU line can never silently
    claim GPUs it did not run on."""
    if n_devices < 1:
        raise ValueError("no visible GPU")
    if local_world > n_devices and not share:
        raise ValueError(f"{local_world} ranks on this node but only {n_devices} visible GPU(s); pass --share-gpus "
                         "to let ranks share devices (the line then says so)")
    return local_rank % n_devices


def local_world_size(env: "DistEnv") -> int:
    """Ranks on this node: LOCAL_WORLD_SIZE (torch.distributed.run and
    spawn_ranks set it), else the whole world (a one-node job)."""
    return int(os.environ.get("LOCAL_WORLD_SIZE", env.world))


def timed_steps(env: "DistEnv", steps: int, step, sync, before_start=None) -> tuple[int, int]:
    """The timed region of one rank: sync + barrier, then ``step(i)`` for i < steps,
    then sync, bracketed by this rank's start and end on CLOCK_MONOTONIC (ns),
    which every process of the node shares, so ranks' times compare directly.
    ``before_start`` runs between the barrier and the start (tests inject a
    start skew there)."""
    sync()
    barrier(env)
    if before_start is not None:
        before_start()
    t0 = time.monotonic_ns()
    for i in range(steps):
        step(i)
    sync()
    t1 = time.monotonic_ns()
    barrier(env)
    return t0, t1


def aggregate(starts_ns, ends_ns, units, steps: int) -> dict:
    """SURVEY.md 8e's aggregate over ranks that share one clock: Σ units x steps
    / (latest end - earliest start).  A rank that starts late after the barrier
    lengthens the span, so the rate cannot be overstated by start skew; the
    max-over-ranks elapsed time (each rank's own end - start) is kept beside it."""
    span = max(ends_ns) - min(starts_ns)
    own = [e - s for s, e in zip(starts_ns, ends_ns)]
    total = float(sum(units)) * steps
    return {"span_s": span / 1e9, "max_rank_s": max(own) / 1e9,
            "start_skew_ms": (max(starts_ns) - min(starts_ns)) / 1e6,
            "end_skew_ms": (max(ends_ns) - min(ends_ns)) / 1e6,
            "rate": total / (span / 1e9), "rate_max_rank": total / (max(own) / 1e9)}


def init_control_plane(env: DistEnv) -> None:
    """gloo process group for the barrier and the MAX of elapsed times."""
    if not env.distributed:
        return
    import torch.distributed as dist

    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=env.rank, world_size=env.world)


def barrier(env: DistEnv) -> None:
    if env.distributed:
        import torch.distributed as dist

        dist.barrier()


def max_over_ranks(env: DistEnv, value: float) -> float:
    if not env.distributed:
        return value
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(env: DistEnv, value: float) -> float:
    if not env.distributed:
        return value
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def gather_over_ranks(env: DistEnv, values: list[float]) -> list[list[float]]:
    """Every rank's ``values`` (same length on all ranks), indexed by rank."""
    if not env.distributed:
        return [list(values)]
    import torch
    import torch.distributed as dist

    t = torch.tensor(values, dtype=torch.float64)
    out = [torch.empty_like(t) for _ in range(env.world)]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]


def gather_ints(env: DistEnv, values: list[int]) -> list[list[int]]:
    """Every rank's int64 ``values`` (exact: clock readings in ns), indexed by rank."""
    if not env.distributed:
        return [[int(v) for v in values]]
    import torch
    import torch.distributed as dist

    t = torch.tensor(values, dtype=torch.int64)
    out = [torch.empty_like(t) for _ in range(env.world)]
    dist.all_gather(out, t)
    return [[int(x) for x in o.tolist()] for o in out]


def gather_objects(env: DistEnv, obj) -> list:
    """Every rank's picklable ``obj`` (small control records), indexed by rank."""
    if not env.distributed:
        return [obj]
    import torch.distributed as dist

    out = [None] * env.world
    dist.all_gather_object(out, obj)
    return out


def shutdown(env: DistEnv) -> None:
    if env.distributed:
        import torch.distributed as dist

        if dist.is_initialized():
            dist.destroy_process_group()

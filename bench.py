#!/usr/bin/env python3
"""Headline benchmark: device-resident MTU-9000 TCP checksum batches (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload cfg5]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

With ``--gpus N > 1`` and no WORLD_SIZE in the environment, bench.py starts
the N ranks itself (one child process per GPU, ``shard.spawn_ranks``; the
parent never touches the GPU).  Under torch.distributed.run, WORLD_SIZE must
equal --gpus.

A step = one launch of the checksum kernel over this rank's whole shard of
synthetic packets already resident in HBM (generated on the device from
global packet ids; cfg5 = 8,980-byte TCP/IPv4 segments, 8M packets per GPU,
64M at 8 GPUs -> weak scaling).  Ranks share nothing on the data path: fixed
configs split the global packet-id range evenly, ragged ones (cfg4) at equal
L4 bytes.  gloo carries the barrier, every rank's start and end on the
node's shared monotonic clock and the per-rank figures.  Rank 0 prints ONE
JSON line.

value   = checksummed L4 bytes of all ranks x K / (latest end - earliest start)
          over ranks, GiB/s; the max-over-ranks elapsed time and
          the start skew after the barrier are reported beside it
roofline: algorithmic bytes per launch (L + 2 per packet: L read, u16 written)
          / the MEDIAN per-dispatch duration (a HIP event pair around every
          launch, on the launch stream), vs 8 TB/s; the back-to-back mean is
          reported beside it
cpu_baseline: pip's own pip_inet_checksum / pip_ip_checksum (oracle/_ref,
          compiled from the reference) -- or the oracle's C restatement if
          _ref is absent -- on a bounded sample of the same packets, all host
          cores and one core; rank 0, N=1.  Beside it ("chain"): the call pip's
          TX path makes, pip_inet{,6}_checksum_buf on a header -> payload
          pip_buf chain, over the same sample.
roofline.traffic: PMC HBM bytes per launch from profiles/traffic_<cfg>.json,
          attached only when that file was measured on the same kernel
          instantiation (pipck_last_launch) of the same libpipck.so (sha256).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402

from pip_amd import shard  # noqa: E402
from pip_amd._lib import HDR_TCP, HDR_UDP  # noqa: E402
from pip_amd.workloads import ALL, BY_CFG, N_FLOWS  # noqa: E402

METRIC = "GiB/s payload checksummed (device-resident), MTU-9000 TCP batch; Mpkt/s"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
PER_GPU_PACKETS = 8 << 20  # cfg5: 64M packets over 8 GPUs
LAUNCH_BOUND_S = 50e-6  # below this an event pair costs as much as the kernel (cfg1 at 1M headers)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    # the GPU's clocks ramp for ~25 ms of work after an idle gap (profiles/
    # r04_ramp.jsonl): 40 warmup launches cover it for every config (cfg2-4 run
    # ~1 ms per launch; the driver's --warmup 5 already covers cfg5's 10 ms)
    p.add_argument("--warmup", type=int, default=40)
    p.add_argument("--workload", default="cfg5", help="cfg1..cfg5 (default: the headline cfg5)")
    p.add_argument("--packets-per-gpu", type=int, default=0, help="override the per-GPU shard size")
    p.add_argument("--cpu-sample", type=int, default=0, help="packets in the CPU-baseline sample (0 = auto)")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline and host end-to-end legs")
    p.add_argument("--results-host", action="store_true",
                   help="write the 2-B results straight into pinned host memory (where pip consumes them) instead "
                        "of HBM; the batch stays in HBM; the line says so and carries no PMC traffic figure")
    p.add_argument("--traffic", default="auto",
                   help="JSON with PMC-measured HBM bytes per launch (auto: profiles/traffic_<workload>.json); "
                        "attached only if measured on this exact kernel of this exact libpipck.so build")
    p.add_argument("--tune", default="",
                   help="measurement only: JSON of engine.tune kwargs (internal launch-shape override); "
                        "the line then names it in config.tune_override")
    p.add_argument("--start-skew-ms", type=float, default=0.0,
                   help="rehearsal/test only: rank r waits r x this after the barrier before its timed start")
    p.add_argument("--digest", action="store_true",
                   help="add per_rank_results: each rank's shard (first packet id, count) and the sha256 of its "
                        "u16 results, after the timed region (multi-rank rehearsals compare them with one-rank runs)")
    p.add_argument("--share-gpus", action="store_true",
                   help="allow more ranks than visible GPUs (ranks then share devices; rehearsal only)")
    return p.parse_args(argv)


def lib_sha256() -> str:
    import hashlib

    from pip_amd import _lib

    return hashlib.sha256(Path(_lib.LIBPIPCK).read_bytes()).hexdigest()


def last_kernel() -> str:
    """The exact kernel instantiation the last batch launch on this thread ran (pipck_last_launch)."""
    import ctypes as C

    from pip_amd import _lib

    buf = C.create_string_buffer(4096)
    _lib.check("pipck_last_launch", _lib.load().pipck_last_launch(buf, len(buf)))
    return buf.value.decode()


class HipEvents:
    """n timing events of the HIP runtime already mapped into the process (the
    one libpipck launches through, engine.hip_runtime), recorded on one stream
    by raw hipEventRecord."""

    def __init__(self, n: int, stream: int | None):
        import ctypes as C

        self._C = C
        # RTLD_NOLOAD: a handle on the mapped instance, never a fresh load
        from pip_amd import engine

        self.hip = engine.hip_runtime()
        self.hip.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
        self.hip.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
        self.hip.hipEventDestroy.argtypes = [C.c_void_p]
        self.stream = C.c_void_p(stream)
        self.ev = [C.c_void_p() for _ in range(n)]
        for e in self.ev:
            if self.hip.hipEventCreate(C.byref(e)) != 0:
                raise RuntimeError("hipEventCreate failed")
        self._rec = self.hip.hipEventRecord

    def record(self, i: int) -> None:
        if self._rec(self.ev[i], self.stream) != 0:
            raise RuntimeError("hipEventRecord failed")

    def elapsed_s(self, a: int, b: int) -> float:
        ms = self._C.c_float()
        if self.hip.hipEventElapsedTime(self._C.byref(ms), self.ev[a], self.ev[b]) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        return ms.value / 1e3

    def destroy(self) -> None:
        for e in self.ev:
            self.hip.hipEventDestroy(e)
        self.ev = []


def match_traffic(t: dict, kernel: str, lib_sha: str, algo_bytes: int, stride: int):
    """A PMC traffic record applies to a bench line only if it was measured on the
    same kernel instantiation (full demangled name), the same library build
    (sha256 of libpipck.so), the same per-launch byte count and layout.
    Returns (hbm bytes per launch or None, reason)."""
    checks = (("kernel", t.get("kernel") == kernel), ("lib_sha256", t.get("lib_sha256") == lib_sha),
              ("algorithmic_bytes_per_launch", t.get("algorithmic_bytes_per_launch") == algo_bytes),
              ("arena_stride", t.get("arena_stride") == stride))
    bad = [name for name, ok in checks if not ok]
    if bad:
        return None, "mismatch: " + ", ".join(bad)
    return t.get("hbm_bytes_per_launch"), "match"


def host_threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(n, cap) if cap else n)


def workload(name: str):
    return ALL[name] if name in ALL else BY_CFG[int(name.lstrip("cfg"))]


def main(argv=None) -> int:
    args = parse(argv)
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr)
        return 2
    if "WORLD_SIZE" in os.environ:
        if int(os.environ["WORLD_SIZE"]) != args.gpus:
            print(f"bench.py: WORLD_SIZE={os.environ['WORLD_SIZE']} but --gpus {args.gpus}", file=sys.stderr)
            return 2
    elif args.gpus > 1:
        # one process per GPU; this parent process never initialises HIP
        return shard.spawn_ranks(args.gpus, [sys.executable, os.path.abspath(__file__), *sys.argv[1:]])
    return run_rank(args)


def run_rank(args) -> int:
    env = shard.dist_env()
    shard.init_control_plane(env)

    import torch

    from pip_amd import engine

    # one GPU per rank; more ranks than visible GPUs only with --share-gpus (a
    # rehearsal), and never silently: the line then says the GPUs were shared
    n_dev = torch.cuda.device_count()
    try:
        dev = shard.device_for_rank(env.local_rank, shard.local_world_size(env), n_dev, args.share_gpus)
    except ValueError as e:
        print(f"bench.py: {e}", file=sys.stderr)
        shard.shutdown(env)
        return 3
    torch.cuda.set_device(dev)
    engine.require_gpu()
    if args.tune:
        engine.tune(**json.loads(args.tune))
    import socket

    placement = {"rank": env.rank, "host": socket.gethostname(), "device": dev, "pci_bus_id": engine.pci_bus_id(dev),
                 "name": torch.cuda.get_device_name(dev)}
    w = workload(args.workload)
    per_gpu = args.packets_per_gpu or (PER_GPU_PACKETS if w.cfg == 5 else w.n_packets)

    def host_out(count):  # --results-host: the kernel's result stores go to pinned host memory
        return torch.empty(count, dtype=torch.int16, pin_memory=True) if args.results_host else None
    n_total = per_gpu * env.world

    # ---- this rank's shard, generated in HBM from global packet ids
    pseudo = engine.gen_flows(w.family, N_FLOWS, w.seed, w.proto)[1] if w.family else None
    if w.ragged:
        # ragged: contiguous ranges of equal L4 bytes, cut on the
        # prefix of every packet's length -- the same on every rank
        if env.world > 1:
            lens_all = torch.empty(n_total, dtype=torch.int32, device="cuda")
            engine.call("pipck_gen_zipf_lengths", engine._ptr(lens_all), n_total, 0, w.seed,
                        engine.current_stream())
            prefix = torch.zeros(n_total + 1, dtype=torch.int64, device="cuda")
            torch.cumsum(lens_all.to(torch.int64), 0, out=prefix[1:])
            cuts = shard.byte_cuts(prefix, env.world)
            first, count = cuts[env.rank], cuts[env.rank + 1] - cuts[env.rank]
            lens = lens_all[first:first + count].clone()
            del lens_all, prefix
        else:
            first, count, lens = 0, n_total, None
        # the byte-packed layout: packets back to back with no padding, u16
        # lengths + one u64 byte offset per 64 packets instead of 16-byte descriptors
        arena, lens16, tile_off, lens = engine.gen_packed_bytes(count, first, w.seed, w.hdr, lengths=lens)
        l4_bytes = int(lens.to(torch.int64).sum().item())

        # the C ABI call bound once (pointers, sizes, stream): a step costs the host
        # what a C caller pays, not this package's per-call argument handling
        step, out = engine.prepare_checksum_packed_bytes(arena, lens16, tile_off, count, pseudo, N_FLOWS, None, first,
                                                         out=host_out(count))
    else:
        first, count = shard.shard_range(n_total, env.world, env.rank)
        arena = torch.empty(count * w.stride, dtype=torch.uint8, device="cuda")
        engine.gen_fixed(arena, w.stride, w.length, count, first, w.seed, w.hdr)
        l4_bytes = count * w.length

        step, out = engine.prepare_checksum_fixed(arena, w.stride, w.length, count, pseudo, N_FLOWS, None, first,
                                                  out=host_out(count))
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()

    # a HIP event pair around every launch, on the launch stream (engine launches
    # on torch's current stream): per-dispatch durations without a profiler.  Raw
    # hipEventRecord through ctypes: torch.cuda.Event.record costs ~6 us of host
    # time per event, which on a launch-bound batch (cfg1's 1M headers) is more
    # than the kernel, and it inflated that kernel's event-pair median from 7.0
    # to 8.4 us (tools/call_overhead.py, profiles/r05_call_overhead.jsonl)
    ev = HipEvents(2 * args.steps, engine.current_stream().value)

    def timed_step(i):
        ev.record(2 * i)
        step()
        ev.record(2 * i + 1)

    skew = (lambda: time.sleep(env.rank * args.start_skew_ms / 1e3)) if args.start_skew_ms else None
    t0, t1 = shard.timed_steps(env, args.steps, timed_step, torch.cuda.synchronize, before_start=skew)
    kernel = last_kernel()  # the instantiation the timed launches ran
    per_launch = sorted(ev.elapsed_s(2 * i, 2 * i + 1) for i in range(args.steps))
    launch_s = per_launch[len(per_launch) // 2] if args.steps % 2 else \
        (per_launch[args.steps // 2 - 1] + per_launch[args.steps // 2]) / 2
    b2b_s = ev.elapsed_s(0, 2 * args.steps - 1) / args.steps
    ev.destroy()
    ranks = shard.gather_over_ranks(env, [float(l4_bytes), float(count), (t1 - t0) / 1e9, launch_s])
    clocks = shard.gather_ints(env, [t0, t1])
    placements = shard.gather_objects(env, placement)
    digests = None
    if args.digest:  # after the timed region: the results of this rank's shard
        import hashlib

        res = out.cpu().numpy().tobytes()
        digests = shard.gather_objects(env, {"rank": env.rank, "first": int(first), "count": int(count),
                                             "sha256": hashlib.sha256(res).hexdigest()})
    total_bytes = sum(r[0] for r in ranks)
    total_pkts = sum(r[1] for r in ranks)
    one_host = len({p["host"] for p in placements}) == 1
    agg = shard.aggregate([c[0] for c in clocks], [c[1] for c in clocks], [r[0] for r in ranks], args.steps)
    # ranks on one node share CLOCK_MONOTONIC: the span from the earliest start to
    # the latest end; across nodes the clocks differ and only each
    # rank's own elapsed time is comparable
    elapsed = agg["span_s"] if one_host else agg["max_rank_s"]

    gib_s = total_bytes * args.steps / elapsed / 2**30
    # L4 payload only: the checksummed bytes minus the TCP (20 B) /
    # UDP (8 B) header of every packet; an IPv4-header batch (cfg1) has none
    hdr_len = {HDR_TCP: 20, HDR_UDP: 8}.get(w.hdr, 0)
    payload_gib_s = (total_bytes - hdr_len * total_pkts) * args.steps / elapsed / 2**30
    mpkt_s = total_pkts * args.steps / elapsed / 1e6
    algo_bytes = l4_bytes + 2 * count  # per launch on this rank
    achieved = algo_bytes / launch_s / 1e9
    traffic, traffic_src, rocprof_ms = None, "none", None
    sha = lib_sha256()
    tpath = Path(args.traffic) if args.traffic != "auto" else ROOT / "profiles" / f"traffic_cfg{w.cfg}.json"
    if args.results_host:
        traffic_src = "none (--results-host: the profiles' PMC passes wrote the results to HBM)"
    elif args.traffic and tpath.exists():
        t = json.loads(tpath.read_text())
        traffic, why = match_traffic(t, kernel, sha, algo_bytes, w.stride)
        traffic_src = f"{tpath.relative_to(ROOT) if tpath.is_relative_to(ROOT) else tpath} ({why})"
        if traffic is not None and t.get("rocprof_timed_median_ns"):
            rocprof_ms = t["rocprof_timed_median_ns"] / 1e6
    launch_bound = launch_s < LAUNCH_BOUND_S
    n_shared = env.world - len({(p["host"], p["pci_bus_id"]) for p in placements})

    line = {
        "metric": METRIC,
        "value": round(gib_s, 2),
        "unit": "GiB/s",
        "n_gpus": env.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: device-generated counter-hash packets (0.1% all-zero, 0.1% all-0xFF), 1024 flows",
        "config": {
            "workload": f"{w.name}: {w.describe(int(total_pkts), env.world)}",
            "packets_per_gpu": count,
            "global_packets": int(total_pkts),
            "l4_bytes_per_packet": w.length,
            "arena_stride": w.stride,
            "layout": "byte-packed (no padding), u16 lengths + u64 byte offset per 64 packets" if w.ragged
                      else f"fixed {w.stride}-byte slots",
            **({"tune_override": json.loads(args.tune)} if args.tune else {}),
            "results": "pinned host memory (--results-host)" if args.results_host else "HBM",
            "parallelism": f"{env.world} shard(s), contiguous packet ranges"
                           f"{' of equal bytes' if w.ragged else ''}, no data-path collective"
                           f"{f', {env.world} ranks SHARING {env.world - n_shared} GPU(s) (--share-gpus)' if n_shared else ''}",
        },
        "mpkt_per_s": round(mpkt_s, 2),
        "per_gpu_gib_per_s": round(gib_s / env.world, 2),
        # each rank's own rate over its own wall time and shard
        "per_rank_gib_per_s": [round(r[0] * args.steps / r[2] / 2**30, 2) for r in ranks],
        "per_rank_packets": [int(r[1]) for r in ranks],
        "timing": {
            "value_over": "latest end - earliest start over ranks (one node's monotonic clock)" if one_host
                          else "max over ranks of each rank's own elapsed time (ranks on several hosts)",
            "span_ms": round(agg["span_s"] * 1e3, 4),
            "max_rank_elapsed_ms": round(agg["max_rank_s"] * 1e3, 4),
            "start_skew_ms": round(agg["start_skew_ms"], 4),
            "end_skew_ms": round(agg["end_skew_ms"], 4),
            "value_by_max_rank_elapsed": round(agg["rate_max_rank"] / 2**30, 2),
            "injected_start_skew_ms_per_rank": args.start_skew_ms or None,
        },
        "devices_visible": n_dev,
        "distinct_gpus": env.world - n_shared,
        "per_rank_device": placements,
        "l4_payload_gib_per_s": round(payload_gib_s, 2),
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "kernel_ms": round(launch_s * 1e3, 4),
            "kernel_ms_b2b_mean": round(b2b_s * 1e3, 4),
            "kernel_ms_min": round(per_launch[0] * 1e3, 4),
            "timing": "median of per-dispatch HIP event pairs on the launch stream",
            "algorithmic_bytes_per_launch": algo_bytes,
            "kernel": kernel,
            "lib_sha256": sha,
            "traffic_source": traffic_src,
            "launch_bound": launch_bound,
        },
        "cpu_baseline": None,
    }
    if digests is not None:
        line["per_rank_results"] = digests
    if launch_bound:
        # sub-50 us launches: the event pair and launch cost as much as the kernel;
        # the rocprof trace of the same kernel and build is the kernel's own duration
        line["roofline"]["timing"] += "; LAUNCH-BOUND at this size (kernel < 50 us): frac reflects launch overhead"
        if rocprof_ms:
            line["roofline"]["rocprof_kernel_ms"] = round(rocprof_ms, 5)
            line["roofline"]["frac_rocprof"] = round(algo_bytes / (rocprof_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)

    if env.rank == 0 and env.world == 1 and not args.no_cpu:
        dev = (arena, lens16, tile_off) if w.ragged else None
        line["cpu_baseline"], line["host_end_to_end"] = cpu_legs(args, w, out, count, first, dev)

    shard.barrier(env)
    if env.rank == 0:
        print(json.dumps(line), flush=True)
    shard.shutdown(env)
    return 0


def _timed(run, threads, budget_s=3.0, max_reps=50):
    """Repeat run(threads) for about budget_s; return (reps, seconds)."""
    reps, t0 = 0, time.perf_counter()
    while True:
        run(threads)
        reps += 1
        el = time.perf_counter() - t0
        if el > budget_s or reps >= max_reps:
            return reps, el


def chain_leg(ref, w, arena, offs, lens, flows, first, threads, want):
    """pip's TX call itself: pip_inet{,6}_checksum_buf on a header pip_buf chained to the payload
    pip_buf (pip_tcp_packet.cpp:28-37 builds it, :124-134 checksums it; pip_udp.cpp the same with
    8 bytes), over the same sample -- beside the flat pip_inet_checksum baseline."""
    if ref is None or not w.family:
        return None
    hdr_len = {HDR_TCP: 20, HDR_UDP: 8}.get(w.hdr, 0)
    chains = ref.tx_chains(arena, offs, lens, hdr_len)
    try:
        def run(t):
            return chains.checksum(w.family, w.proto, flows, N_FLOWS, first, t)

        ok = bool(np.array_equal(run(threads), want))
        reps, el = _timed(run, threads)
        reps1, el1 = _timed(run, 1, budget_s=1.0, max_reps=20)
    finally:
        chains.close()
    l4 = int(lens.astype(np.int64).sum())
    return {"call": f"pip_inet{'6' if w.family == 6 else ''}_checksum_buf on a {hdr_len}-B header pip_buf -> payload "
                    "pip_buf chain, as pip's TX path builds and checksums it (pip_tcp_packet.cpp:28-37, 124-134; "
                    "pip_checksum.cpp:90-148)",
            "value": round(l4 * reps / el / 2**30, 3), "unit": "GiB/s", "cores": threads,
            "single_core_gib_per_s": round(l4 * reps1 / el1 / 2**30, 3),
            "mpkt_per_s": round(len(lens) * reps / el / 1e6, 2), "results_match_flat": ok}


def host_e2e_packed(w, dev, n, flows, want):
    """PCIe-inclusive rate of the first n packets of a byte-packed ragged batch:
    pinned host bytes + lengths -> pipck_host_checksum_packed_bytes (chunks H2D,
    index, k_packedb, D2H) -> host results, checked against the GPU's."""
    import ctypes as C

    import torch

    from pip_amd import _lib

    arena, lens16, tile_off = dev
    del tile_off
    nb = int((lens16[:n].to(torch.int32) & 0xFFFF).sum().item())  # lengths are u16 stored as int16
    h = torch.empty(max(nb, 1), dtype=torch.uint8, pin_memory=True)
    h[:nb].copy_(arena[:nb])
    hl = lens16[:n].cpu().numpy().view(np.uint16).copy()
    out = np.zeros(n, dtype=np.uint16)
    lib = _lib.load()
    ctx = C.c_void_p()
    _lib.check("pipck_ctx_create", lib.pipck_ctx_create(-1, C.byref(ctx)))
    fl = C.create_string_buffer(flows, max(len(flows), 1))
    try:
        call = lambda: lib.pipck_host_checksum_packed_bytes(  # noqa: E731
            ctx, C.c_void_p(h.data_ptr()), C.c_void_p(hl.ctypes.data), n, w.family, fl, N_FLOWS, 0,
            C.c_void_p(out.ctypes.data))
        _lib.check("pipck_host_checksum_packed_bytes", call())
        t0 = time.perf_counter()
        for _ in range(3):
            call()
        e2e = nb * 3 / (time.perf_counter() - t0) / 2**30
    finally:
        lib.pipck_ctx_destroy(ctx)
    return {"value": round(e2e, 2), "unit": "GiB/s", "sample_packets": n, "bytes": nb, "pinned": True,
            "call": "pipck_host_checksum_packed_bytes (byte-packed, ~64 MiB chunks, two streams)",
            "results_match": bool(np.array_equal(out, want))}


def mem_available() -> int:
    """MemAvailable of /proc/meminfo in bytes (0 if unreadable)."""
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                if line.startswith("MemAvailable:"):
                    return int(line.split()[1]) * 1024
    except OSError:
        pass
    return 0


def host_bytes_per_packet(w) -> int:
    """Host memory the CPU legs hold per sampled packet: the packet bytes (a fixed
    slot, or cfg4's Zipf mean of ~990 B rounded up), plus the chain leg's two
    pip_buf objects (they point into the same bytes, ref_chains_build), results
    and per-packet metadata."""
    return (w.stride if not w.ragged else 1024) + 256


def sample_that_fits(n: int, per_packet: int) -> int:
    """n, or the largest sample whose host footprint fits half of MemAvailable."""
    avail = mem_available()
    if not avail or n * per_packet <= avail // 2:
        return n
    return max(1 << 12, int(avail // 2 // per_packet))


def cpu_legs(args, w, gpu_out, count, first, dev=None):
    """pip's own checksum on the host cores over a bounded sample of the same
    packets (checked bit-exact against the GPU results), plus the PCIe-inclusive
    host -> device -> host rate of the same sample: pipck_host_checksum_fixed
    for fixed strides, pipck_host_checksum_packed_bytes for the ragged batch."""
    import ctypes as C

    from oracle.oracle import Oracle, Reference
    from pip_amd import _lib

    threads = host_threads()
    orc = Oracle()
    kind = "reference" if Reference.available() else "port"
    ref = Reference() if kind == "reference" else None
    flows = orc.flows_table(w.family, w.seed, N_FLOWS, w.proto) if w.family else b""
    gpu = gpu_out.cpu().numpy().view(np.uint16)

    # the sample BASELINE.md ("Which inputs") prescribes: the full batch for cfg1-cfg4,
    # the first 1M packets for cfg5 (64M x 8,980 B cannot be host-resident) -- up to
    # ~9 GB of host memory (cfg3, cfg5); --cpu-sample overrides it.  A host with too
    # little free memory for that gets the largest sample that fits in half of
    # what is available, and the line's "sample" says so.
    plan = f"BASELINE.md plan: {'first 1M packets of the per-GPU shard' if w.cfg == 5 else 'the full batch'}"
    n_plan = args.cpu_sample or min(count, 1 << 20 if w.cfg == 5 else count)
    n = sample_that_fits(n_plan, host_bytes_per_packet(w))
    if n < n_plan:
        plan += f"; FELL BACK to {n} of {n_plan} packets: {mem_available() >> 20} MiB of host memory available"
    if w.ragged:
        arena, offs, lens = orc.gen_ragged_batch(w.seed, first, n, w.hdr, threads)
        l4 = int(lens.astype(np.int64).sum())

        def run(t):
            if ref:
                return ref.batch_ragged(arena, offs, lens, w.family, w.proto, flows, N_FLOWS, first, t)
            return orc.batch_ragged(arena, offs, lens, w.family, w.proto, w.seed, N_FLOWS, first, t)

        res = run(threads)  # warm + correctness
        verified = bool(np.array_equal(res, gpu[:n]))
        reps, el = _timed(run, threads)
        t0 = time.perf_counter()
        run(1)
        st = l4 / (time.perf_counter() - t0) / 2**30
        cpu = {"value": round(l4 * reps / el / 2**30, 3), "unit": "GiB/s", "cores": threads, "kind": kind,
               "sample": f"first {n} packets of the same Zipf workload ({l4 / 2**30:.2f} GiB of L4 bytes; "
                         f"{plan if not args.cpu_sample or n < n_plan else '--cpu-sample'}), "
                         f"pip_inet_checksum per packet, {reps} timed passes on {threads} threads; "
                         f"1 thread: {st:.3f} GiB/s",
               "single_core_gib_per_s": round(st, 3), "gpu_results_match": verified,
               "chain": chain_leg(ref, w, arena, offs, lens, flows, first, threads, res)}
        e2e = host_e2e_packed(w, dev, n, flows, gpu[:n]) if dev is not None and first == 0 else \
            {"value": None, "note": "host end-to-end: rank 0 of a one-rank run only"}
        return cpu, e2e

    lib = _lib.load()
    pin = lib.pipck_host_alloc(n * w.stride)
    if not pin:
        raise RuntimeError("pipck_host_alloc failed")
    arena = np.ctypeslib.as_array((C.c_uint8 * (n * w.stride)).from_address(pin))
    try:
        orc.lib.ock_gen_fixed_batch(w.seed, first, n, w.length, w.hdr, C.c_void_p(pin), w.stride, threads)

        def run(t):
            if ref:
                return ref.batch_fixed(arena, w.stride, w.length, n, w.family, w.proto, flows, N_FLOWS, first, t)
            return orc.batch_fixed(arena, w.stride, w.length, n, w.family, w.proto, w.seed, N_FLOWS, first, t)

        res = run(threads)  # warm + correctness
        verified = bool(np.array_equal(res, gpu[:n]))
        reps, el = _timed(run, threads)
        mt = n * w.length * reps / el / 2**30
        reps1, el1 = _timed(run, 1, budget_s=1.0, max_reps=20)
        st = n * w.length * reps1 / el1 / 2**30
        chain = chain_leg(ref, w, arena, np.arange(n, dtype=np.uint64) * w.stride, np.full(n, w.length, np.uint32),
                          flows, first, threads, res)

        # host end-to-end: pinned host batch -> H2D -> kernel -> D2H (PCIe-bound)
        ctx = C.c_void_p()
        _lib.check("pipck_ctx_create", lib.pipck_ctx_create(-1, C.byref(ctx)))
        h_out = np.zeros(n, dtype=np.uint16)
        fl = C.create_string_buffer(flows, max(len(flows), 1))
        call = lambda: lib.pipck_host_checksum_fixed(  # noqa: E731
            ctx, C.c_void_p(pin), w.stride, w.length, n, w.family, fl, N_FLOWS, first, C.c_void_p(h_out.ctypes.data))
        _lib.check("pipck_host_checksum_fixed", call())
        t0 = time.perf_counter()
        for _ in range(3):
            call()
        e2e = n * w.length * 3 / (time.perf_counter() - t0) / 2**30
        e2e_ok = bool(np.array_equal(h_out, res))
        lib.pipck_ctx_destroy(ctx)
    finally:
        del arena
        lib.pipck_host_free(pin)
    what = "pip_ip_checksum" if not w.family else f"pip_inet{'6' if w.family == 6 else ''}_checksum"
    cpu = {"value": round(mt, 3), "unit": "GiB/s", "cores": threads, "kind": kind,
           "sample": f"first {n} packets of the same workload ({n * w.length / 2**30:.3f} GiB; "
                     f"{plan if not args.cpu_sample or n < n_plan else '--cpu-sample'}), {what} per packet, "
                     f"{reps} timed passes on {threads} threads; 1 thread: {st:.3f} GiB/s",
           "single_core_gib_per_s": round(st, 3),
           "mpkt_per_s": round(n * reps / el / 1e6, 2), "single_core_mpkt_per_s": round(n * reps1 / el1 / 1e6, 2),
           "gpu_results_match": verified, "chain": chain}
    e2e_d = {"value": round(e2e, 2), "unit": "GiB/s", "sample_packets": n, "pinned": True, "results_match": e2e_ok}
    return cpu, e2e_d


if __name__ == "__main__":
    sys.exit(main())

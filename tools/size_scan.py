#!/usr/bin/env python3
"""Kernel throughput vs batch size for launch-shape arms (engine.tune kwargs).

    python tools/size_scan.py [--iters 10] [--only cfg4] [--sizes 8,32] [--arms '{"a": {...}}']

One JSON line per (workload, packets, arm): median kernel ms (HIP events) and
algorithmic GB/s.  All arms run in one process, interleaved, results checked equal.
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from pip_amd import engine  # noqa: E402
from pip_amd.workloads import BY_CFG, CFG4, CFG5, N_FLOWS  # noqa: E402

DEFAULT_SIZES = {1: (1 << 20,), 2: (4 << 20,), 3: (1 << 20,), 4: (8 << 20, 32 << 20),
                 5: (2 << 20, 4 << 20, 8 << 20, 16 << 20)}


def timed_b2b(fn, iters):
    """bench.py's timing: iters launches back to back (no host sync between
    them), an event pair around each, median per-dispatch time."""
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in ev)


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="", help="comma list of cfgN (default cfg5,cfg4)")
    ap.add_argument("--sizes", default="", help="comma list of packet counts in Mi (default per workload)")
    ap.add_argument("--pseudo", action="store_true", help="fixed-stride workloads: add IPv4 pseudo-headers even for cfg1")
    ap.add_argument("--packed", action="store_true", help="ragged workloads: the 16-B packed-lengths kernel")
    ap.add_argument("--packedb", action="store_true", help="ragged workloads: the byte-packed kernel (bench.py's)")
    ap.add_argument("--arms", default="", help="JSON {arm: engine.tune kwargs}, or @file (default: built-in arms)")
    ap.add_argument("--b2b", action="store_true",
                    help="time launches back to back as bench.py does (default: a host sync after every launch)")
    a = ap.parse_args()
    clock = timed_b2b if a.b2b else timed
    engine.require_gpu()
    plan = [(CFG5, (2 << 20, 4 << 20, 8 << 20, 16 << 20)), (CFG4, (8 << 20, 32 << 20))]
    if a.only:
        cfgs = [int(c.strip().lstrip("cfg")) for c in a.only.split(",")]
        plan = [(BY_CFG[c], DEFAULT_SIZES[c]) for c in cfgs]
    if a.sizes:
        plan = [(w, tuple(int(float(x) * (1 << 20)) for x in a.sizes.split(","))) for w, _ in plan]
    for w, sizes in plan:
        fam = w.family or (4 if a.pseudo else 0)  # cfg1: IP header, no pseudo-header
        pseudo = engine.gen_flows(fam, N_FLOWS, w.seed, w.proto or 6)[1] if fam else None
        for n in sizes:
            if w.ragged and a.packedb:  # the byte-packed layout bench.py runs (u16 lengths + per-64 byte offset)
                arena, lens16, tile_off, lens = engine.gen_packed_bytes(n, 0, w.seed, w.hdr)
                nbytes = int(lens.to(torch.int64).sum().item()) + 2 * n
                run = lambda: engine.checksum_packed_bytes(arena, lens16, tile_off, n, pseudo, N_FLOWS)  # noqa: E731
            elif w.ragged and a.packed:  # the 16-B packed layout (u16 lengths + per-64 index)
                arena, lens16, tile_chunk, lens = engine.gen_packed(n, 0, w.seed, w.hdr)
                nbytes = int(lens.to(torch.int64).sum().item()) + 2 * n
                run = lambda: engine.checksum_packed(arena, lens16, tile_chunk, n, pseudo, N_FLOWS)  # noqa: E731
            elif w.ragged:
                arena, desc, lens = engine.gen_ragged(n, 0, w.seed, w.hdr, N_FLOWS)
                nbytes = int(lens.to(torch.int64).sum().item()) + 2 * n
                run = lambda: engine.checksum_ragged(arena, desc, pseudo)  # noqa: E731
            else:
                arena = torch.empty(n * w.stride, dtype=torch.uint8, device="cuda")
                engine.gen_fixed(arena, w.stride, w.length, n, 0, w.seed, w.hdr)
                nbytes = (w.length + 2) * n
                run = lambda: engine.checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS)  # noqa: E731
            res = {}
            arms = {"default": {}, "loads_8": {"loads_per_lane": 8}, "pipe_8": {"loads_per_lane": 9}, "pipe_4": {"loads_per_lane": 5},
                    "rows_128": {"rows_per_task": 128}}
            if w.ragged:
                arms = {"default": {}, "wide_blocks": {"wide_blocks": True}, "loads_8": {"loads_per_lane": 8},
                        "pipe_4": {"loads_per_lane": 5}, "loads_2": {"loads_per_lane": 2}}
            if a.arms:
                arms = json.loads(Path(a.arms[1:]).read_text() if a.arms.startswith("@") else a.arms)
            for rnd in range(5):
                for xcd, kw in arms.items():
                    engine.tune(**kw)
                    res.setdefault(xcd, []).append(clock(run, a.iters))
                    out = run()
                    if rnd == 0 and xcd == next(iter(arms)):
                        ref = out.clone()
                    elif "probe" not in xcd:  # probe arms (e.g. loads_only) time a kernel that computes nothing
                        assert torch.equal(out, ref)
            for xcd, ms in res.items():
                m = statistics.median(ms)
                print(json.dumps({"workload": w.name, "packets": n, "gbytes": round(nbytes / 1e9, 1), "bytes": nbytes,
                                  "arm": xcd, "ms": round(m, 4), "GBps": round(nbytes / m / 1e6, 1),
                                  "timing": "back to back" if a.b2b else "synced"}),
                      flush=True)
            engine.tune()
            del arena
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

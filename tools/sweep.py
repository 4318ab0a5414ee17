#!/usr/bin/env python3
"""Launch-shape sweep on one GPU: kernel time per (workload, lanes, loads, blocks, nt).

    python tools/sweep.py [--workloads cfg5,cfg2,...] [--iters 10] [--quick]

Prints one JSON line per measurement (median kernel ms over --iters launches,
HIP events on the launch stream) and the GB/s of algorithmic bytes (L + 2 per
packet).  Results are checked against the auto-shape run of the same batch.
"""
from __future__ import annotations

import argparse
import itertools
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from pip_amd import engine  # noqa: E402
from pip_amd.workloads import BY_CFG, N_FLOWS  # noqa: E402

SIZES = {1: 8 << 20, 2: 4 << 20, 3: 1 << 20, 4: 8 << 20, 5: 4 << 20}


def timed(fn, iters):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    fn()
    torch.cuda.synchronize()
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in ev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="cfg5,cfg2,cfg3,cfg4,cfg1")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--flat-only", action="store_true")
    a = ap.parse_args()
    engine.require_gpu()
    for name in a.workloads.split(","):
        w = BY_CFG[int(name.lstrip("cfg"))]
        n = SIZES[w.cfg]
        pseudo = engine.gen_flows(w.family, N_FLOWS, w.seed, w.proto)[1] if w.family else None
        if w.ragged:
            arena, desc, lens = engine.gen_ragged(n, 0, w.seed, w.hdr, N_FLOWS)
            nbytes = int(lens.to(torch.int64).sum().item()) + 2 * n
            run = lambda: engine.checksum_ragged(arena, desc, pseudo)  # noqa: E731
            shapes = [(0, u, b, True) for u in (2, 4, 3, 5) for b in (0, 8192, 32768, 65536)]
            shapes += [(0, 4, 0, False)]
        else:
            arena = torch.empty(n * w.stride, dtype=torch.uint8, device="cuda")
            engine.gen_fixed(arena, w.stride, w.length, n, 0, w.seed, w.hdr)
            nbytes = (w.length + 2) * n
            run = lambda: engine.checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS)  # noqa: E731
            lanes = [8, 32] if a.quick else [1, 2, 4, 8, 16, 32, 64]
            blocks = [0, 4096] if a.quick else [0, 1024, 4096]
            shapes = [] if a.flat_only else [(g, 0, b, nt) for g, b, nt in itertools.product(lanes, blocks, (False, True))]
            # the flat-stream kernel (lanes 0 = automatic): rows in flight (3/5/9 = pipelined 2/4/8) x grid x policy
            shapes += [(0, u, b, nt) for u, b, nt in itertools.product((8, 16, 9), (0, 16384, 32768), (False, True))]
            shapes += [(0, u, 0, True, r) for u in (8, 16) for r in (16, 64, 128, 256)]
        engine.tune()
        ref = run().clone()
        for shape in shapes:
            g, u, b, nt = shape[:4]
            rows = shape[4] if len(shape) > 4 else 0
            engine.tune(g, u, b, plain_loads=not nt, nt_loads=nt, flat=(g == 0), rows_per_task=rows)
            ms = timed(run, a.iters)
            ok = bool(torch.equal(run(), ref))
            print(json.dumps({"workload": w.name, "lanes": g, "loads": u, "blocks": b, "nt": nt, "rows": rows,
                              "ms": round(ms, 4),
                              "GBps": round(nbytes / ms / 1e6, 1), "ok": ok}), flush=True)
        engine.tune()
        del arena
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Placement probe for the IPv4-header kernel (k_hdr, cfg1 at 256M headers):
the same batch timed with its result array allocated before / after the arena
and at several offsets, to see whether where the 2-byte result stream lands
relative to the read stream moves the rate (a 0.88 vs 0.98 ms bimodality was
seen once in profiles/r03_hdr_scan.jsonl).  One JSON line per arm; results
checked equal.

    python tools/hdr_placement.py [--n 268435456] [--rounds 3]
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
from pip_amd.workloads import CFG1  # noqa: E402
from tools.size_scan import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256 << 20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    engine.require_gpu()
    w, n = CFG1, a.n
    MB = 1 << 20
    arms = {}
    # out allocated first, then the arena
    pool_first = torch.empty(2 * n + 512 * MB, dtype=torch.uint8, device="cuda")
    arena = torch.empty(n * w.stride, dtype=torch.uint8, device="cuda")
    engine.gen_fixed(arena, w.stride, w.length, n, 0, w.seed, w.hdr)
    pool_after = torch.empty(2 * n + 512 * MB, dtype=torch.uint8, device="cuda")
    for name, pool in (("before", pool_first), ("after", pool_after)):
        for off in (0, 4096, 64 * 1024, 2 * MB, 96 * MB, 256 * MB + 4096):
            arms[f"out_{name}_off{off}"] = pool[off:off + 2 * n].view(torch.int16)
    res = {}
    ref = None
    for _ in range(a.rounds):
        for k, out in arms.items():
            fn = lambda: engine.checksum_fixed(arena, w.stride, w.length, n, None, 1, None, 0, out=out)  # noqa: E731
            res.setdefault(k, []).append(timed(fn, 10))
            if ref is None:
                ref = out.clone()
            else:
                assert torch.equal(out, ref), k
    nbytes = (w.length + 2) * n
    for k, ms in res.items():
        m = statistics.median(ms)
        print(json.dumps({"workload": w.name, "packets": n, "arm": k, "ms": round(m, 4),
                          "GBps": round(nbytes / m / 1e6, 1), "rounds_ms": [round(x, 4) for x in ms],
                          "out_minus_arena_mb": round((arms[k].data_ptr() - arena.data_ptr()) / MB, 3)}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""cfg5 at the full per-GPU batch (8M packets, 75 GB): grid x task-size scan of
the flat-stream kernel.  One JSON line per arm; median of 3 interleaved rounds."""
from __future__ import annotations

import itertools
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from pip_amd import engine  # noqa: E402
from pip_amd.workloads import CFG5, N_FLOWS  # noqa: E402

sys.path.insert(0, str(Path(__file__).resolve().parent))
from split_scan import timed  # noqa: E402


def main():
    engine.require_gpu()
    w, n = CFG5, int(sys.argv[1]) if len(sys.argv) > 1 else 8 << 20
    _, pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)
    arena = torch.empty(n * w.stride, dtype=torch.uint8, device="cuda")
    engine.gen_fixed(arena, w.stride, w.length, n, 0, w.seed, w.hdr)
    run = lambda: engine.checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS)  # noqa: E731
    ref = run().clone()
    arms = list(itertools.product((16384, 65536, 131072, 1 << 30), (32, 64, 128, 256)))
    res = {}
    for _ in range(3):
        for blocks, rows in arms:
            engine.tune(blocks=blocks, rows_per_task=rows)
            res.setdefault((blocks, rows), []).append(timed(run, 5))
            assert torch.equal(run(), ref)
    engine.tune()
    nbytes = (w.length + 2) * n
    for (blocks, rows), ms in sorted(res.items(), key=lambda kv: statistics.median(kv[1])):
        m = statistics.median(ms)
        print(json.dumps({"packets": n, "blocks": blocks, "rows": rows, "ms": round(m, 4),
                          "GBps": round(nbytes / m / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""cfg4 layouts in ONE process, timings interleaved: the 16-B-granular packed
layout (k_packed) vs the byte-packed one (k_packedb) over the same packets,
results checked equal.  One JSON line per (packets, layout).

    python tools/layout_ab.py [--sizes 8,16] [--rounds 7] [--iters 10]
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
from pip_amd.workloads import CFG4, N_FLOWS  # noqa: E402
from tools.size_scan import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="8,16")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    engine.require_gpu()
    w = CFG4
    _, pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)
    for m in a.sizes.split(","):
        n = int(float(m) * (1 << 20))
        a16, l16, tc, lens = engine.gen_packed(n, 0, w.seed, w.hdr)
        ab, lb, to, _ = engine.gen_packed_bytes(n, 0, w.seed, w.hdr, lengths=lens)
        nbytes = int(lens.to(torch.int64).sum().item()) + 2 * n
        runs = {"packed16": lambda: engine.checksum_packed(a16, l16, tc, n, pseudo, N_FLOWS),
                "packed_bytes": lambda: engine.checksum_packed_bytes(ab, lb, to, n, pseudo, N_FLOWS)}
        assert torch.equal(runs["packed16"](), runs["packed_bytes"]())
        res = {k: [] for k in runs}
        for _ in range(a.rounds):
            for k, fn in runs.items():
                res[k].append(timed(fn, a.iters))
        for k, ms in res.items():
            med = statistics.median(ms)
            print(json.dumps({"workload": w.name, "packets": n, "layout": k, "ms": round(med, 4),
                              "GBps": round(nbytes / med / 1e6, 1), "rounds_ms": [round(x, 4) for x in ms]}),
                  flush=True)
        del a16, ab
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Flat-stream kernel throughput on cfg2/cfg3/cfg5 at their bench sizes, per
row depth, interleaved rounds in one process (results checked equal).

    python tools/flat_scan.py
"""
from __future__ import annotations

import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from pip_amd import engine  # noqa: E402
from pip_amd.workloads import CFG2, CFG3, CFG5, N_FLOWS  # noqa: E402
from size_scan import timed  # noqa: E402


def main():
    engine.require_gpu()
    for w, n in ((CFG2, 4 << 20), (CFG3, 1 << 20), (CFG5, 8 << 20)):
        pseudo = engine.gen_flows(w.family, N_FLOWS, w.seed, w.proto)[1]
        arena = torch.empty(n * w.stride, dtype=torch.uint8, device="cuda")
        engine.gen_fixed(arena, w.stride, w.length, n, 0, w.seed, w.hdr)
        nbytes = (w.length + 2) * n
        run = lambda: engine.checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS)  # noqa: E731
        arms = {"default": {}, "u8": {"loads_per_lane": 8}, "u16": {"loads_per_lane": 16},
                "pipe8": {"loads_per_lane": 9}, "u4": {"loads_per_lane": 4}}
        res, ref = {}, None
        for _ in range(5):
            for k, kw in arms.items():
                engine.tune(**kw)
                res.setdefault(k, []).append(timed(run, 10))
                out = run()
                if ref is None:
                    ref = out.clone()
                assert torch.equal(out, ref), k
        engine.tune()
        for k, ms in res.items():
            m = statistics.median(ms)
            print(json.dumps({"workload": w.name, "packets": n, "arm": k, "ms": round(m, 4),
                              "GBps": round(nbytes / m / 1e6, 1)}), flush=True)
        del arena
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-launch time series of cfg2's two fixed-stride schedules after an idle
gap: how many launches does each need before it reaches its steady rate?
(bench.py's default warmup must cover the slower one.)  One JSON line per
(trial, schedule): per-launch ms in launch order."""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from pip_amd import engine  # noqa: E402
from pip_amd.workloads import CFG2, N_FLOWS  # noqa: E402


def main():
    engine.require_gpu()
    w, n = CFG2, CFG2.n_packets
    pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)[1]
    arena = torch.empty(n * w.stride, dtype=torch.uint8, device="cuda")
    engine.gen_fixed(arena, w.stride, w.length, n, 0, w.seed, w.hdr)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    launches = int(sys.argv[1]) if len(sys.argv) > 1 else 80
    gap = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    scheds = [("k_flat_coop", {}), ("k_flat", {"alt_flat_schedule": True})]
    for trial in range(3):
        for sname, kw in (scheds if trial % 2 == 0 else scheds[::-1]):
            engine.tune(**kw)
            torch.cuda.synchronize()
            time.sleep(gap)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(launches)]
            for a, b in ev:
                a.record()
                engine.checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS, out=out)
                b.record()
            torch.cuda.synchronize()
            engine.tune()
            print(json.dumps({"trial": trial, "schedule": sname, "gap_s": gap,
                              "ms": [round(a.elapsed_time(b), 4) for a, b in ev]}), flush=True)


if __name__ == "__main__":
    main()

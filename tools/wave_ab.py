#!/usr/bin/env python3
"""The north_star's literal kernel shape -- one packet per wavefront (k_wave,
pipck_wave.hip, tune lanes_per_packet=256) -- against the shipped kernels on
the bench configs, one process, arms interleaved, results compared.

    python tools/wave_ab.py [--only cfg2,cfg3,cfg5,cfg4d] [--rounds 3] [--warm 40]

cfg4d = cfg4's Zipf packets on 16-byte descriptors (pipck_checksum_ragged:
k_ragged vs k_wave); bench.py's cfg4 line runs the byte-packed layout
(k_packedb), reported beside it as cfg4b.  One JSON line per (workload, arm):
median over rounds of the per-round median back-to-back launch time.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))

SIZES = {"cfg2": 4 << 20, "cfg3": 1 << 20, "cfg5": 8 << 20, "cfg4d": 8 << 20, "cfg4b": 8 << 20}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="cfg2,cfg3,cfg5,cfg4d,cfg4b")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warm", type=int, default=40)
    ap.add_argument("--nl", default="0", help="comma list of k_wave loads per lane per pass (0 = auto)")
    a = ap.parse_args()
    import torch

    from pip_amd import engine
    from pip_amd.workloads import BY_CFG, N_FLOWS
    from bench import last_kernel
    from size_scan import timed_b2b

    engine.require_gpu()
    nls = [int(x) for x in a.nl.split(",")]
    for name in a.only.split(","):
        w, n = BY_CFG[int(name[3])], SIZES[name]
        pseudo = engine.gen_flows(w.family, N_FLOWS, w.seed, w.proto or 6)[1] if w.family else None
        if name == "cfg4b":
            arena, lens16, tile_off, lens = engine.gen_packed_bytes(n, 0, w.seed, w.hdr)
            nbytes = int(lens.to(torch.int64).sum().item()) + 2 * n
            out = torch.empty(n, dtype=torch.int16, device="cuda")
            run = lambda: engine.checksum_packed_bytes(arena, lens16, tile_off, n, pseudo, N_FLOWS, None, 0, out=out)  # noqa: E731
            arms = {"shipped": {}}
        elif name == "cfg4d":
            arena, desc, lens = engine.gen_ragged(n, 0, w.seed, w.hdr, N_FLOWS)
            nbytes = int(lens.to(torch.int64).sum().item()) + 2 * n
            run = lambda: engine.checksum_ragged(arena, desc, pseudo)  # noqa: E731
            arms = {"shipped": {}, **{f"wave_nl{x}": {"lanes_per_packet": 256, "loads_per_lane": x} for x in nls}}
        else:
            arena = torch.empty(n * w.stride, dtype=torch.uint8, device="cuda")
            engine.gen_fixed(arena, w.stride, w.length, n, 0, w.seed, w.hdr)
            nbytes = (w.length + 2) * n
            out = torch.empty(n, dtype=torch.int16, device="cuda")
            run = lambda: engine.checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS, None, 0, out=out)  # noqa: E731
            arms = {"shipped": {}, **{f"wave_nl{x}": {"lanes_per_packet": 256, "loads_per_lane": x} for x in nls}}
        res: dict[str, list[float]] = {k: [] for k in arms}
        kern, digest = {}, {}
        for rnd in range(a.rounds):
            order = list(arms.items()) if rnd % 2 == 0 else list(reversed(arms.items()))
            for arm, kw in order:
                engine.tune(**kw)
                try:
                    for _ in range(a.warm):
                        run()
                    res[arm].append(timed_b2b(run, a.iters))
                    kern[arm] = last_kernel()
                    digest[arm] = hashlib.sha256(run().cpu().numpy().tobytes()).hexdigest()[:16]
                finally:
                    engine.tune()
        for arm, ms in res.items():
            m = statistics.median(ms)
            print(json.dumps({"workload": w.name + ("+desc" if name == "cfg4d" else "+bytes" if name == "cfg4b" else ""),
                              "packets": n, "arm": arm, "kernel": kern[arm].split("(")[0], "ms": round(m, 4),
                              "rounds_ms": [round(x, 4) for x in ms], "GBps": round(nbytes / m / 1e6, 1),
                              "frac": round(nbytes / m / 1e6 / 8000, 4),
                              "results_equal_shipped": digest[arm] == digest["shipped"]}), flush=True)
        del arena
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

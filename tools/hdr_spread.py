#!/usr/bin/env python3
"""cfg1's IPv4 headers through k_hdr at 256M headers: the result-stream arms
(VERDICT r03 item 6).

    python tools/hdr_spread.py [--headers N] [--rounds R] [--iters K] [--arms default,in_place]

Arms (one process, interleaved by round, median of K per-launch HIP event
pairs each):
  default   results to a separate u16 array, 16-byte write-through pieces
  in_place  each result stored into its header's ip_sum (tune bit 28): the
            "results inside the headers" layout DESIGN.md r03 speculated about
With --pmc-arm ARM the tool runs that arm a few times only (for one rocprofv3
--pmc pass).  Every line carries the host name, so passes on two boxes can be
told apart.
"""
from __future__ import annotations

import argparse
import json
import socket
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from pip_amd import engine  # noqa: E402
from pip_amd.workloads import CFG1  # noqa: E402

ARMS = {"default": {"loads_per_lane": 32}, "in_place": {"loads_per_lane": 32, "hdr_in_place": True}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--headers", type=int, default=256 << 20)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--arms", default="default,in_place")
    ap.add_argument("--pmc-arm", default="")
    a = ap.parse_args()
    engine.require_gpu()
    w, n = CFG1, a.headers
    arena = torch.empty(n * w.stride, dtype=torch.uint8, device="cuda")
    engine.gen_fixed(arena, w.stride, w.length, n, 0, w.seed, w.hdr)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    run = lambda: engine.checksum_fixed(arena, w.stride, w.length, n, out=out)  # noqa: E731
    algo = n * (w.length + 2)
    host = socket.gethostname()
    if a.pmc_arm:
        engine.tune(**ARMS[a.pmc_arm])
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        engine.tune()
        print(json.dumps({"step": "pmc_pass", "arm": a.pmc_arm, "headers": n, "host": host}), flush=True)
        return
    names = a.arms.split(",")
    med = {k: [] for k in names}
    for r in range(a.rounds):
        for name in (names if r % 2 == 0 else names[::-1]):
            engine.tune(**ARMS[name])
            run()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.iters)]
            for s, e in ev:
                s.record()
                run()
                e.record()
            torch.cuda.synchronize()
            med[name].append(statistics.median(s.elapsed_time(e) for s, e in ev))
            engine.tune()
    summ = {k: round(statistics.median(v), 4) for k, v in med.items()}
    print(json.dumps({"step": "ab", "host": host, "device": torch.cuda.get_device_name(0), "headers": n,
                      "median_ms": summ, "per_round_ms": {k: [round(x, 4) for x in v] for k, v in med.items()},
                      # algorithmic bytes as the bench counts them: 20 B read + 2 B of result per header
                      "frac_of_8TBs": {k: round(algo / (v / 1e3) / 8e12, 4) for k, v in summ.items()}}), flush=True)


if __name__ == "__main__":
    main()

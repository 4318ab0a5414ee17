#!/usr/bin/env python3
"""Fixed-stride schedule arms across strides (engine.tune kwargs), ~6 GB per
stride, arms interleaved by round in one process, results checked equal.

    python tools/stride_scan.py [--strides 1024,1488,2048,3072] [--gbytes 6.2] [--rounds 3] [--arms JSON|@file]

Packets are TCP/IPv4-shaped (cfg2's generator: 20-B header + payload) of
length stride - 8 (so every stride has a masked tail chunk), with IPv4
pseudo-headers.  One JSON line per (stride, arm): median of per-round medians.
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parent))

import torch  # noqa: E402

from pip_amd import engine  # noqa: E402
from pip_amd.workloads import CFG2, N_FLOWS  # noqa: E402
from size_scan import timed  # noqa: E402


def last_kernel() -> str:
    import ctypes as C

    buf = C.create_string_buffer(4096)
    engine.load().pipck_last_launch(buf, len(buf))
    return buf.value.decode().split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--strides", default="1024,1488,2048,3072")
    ap.add_argument("--gbytes", type=float, default=6.2)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=15)
    ap.add_argument("--arms", default='{"default": {}}')
    a = ap.parse_args()
    arms = json.loads(Path(a.arms[1:]).read_text() if a.arms.startswith("@") else a.arms)
    engine.require_gpu()
    w = CFG2
    pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)[1]
    for stride in [int(x) for x in a.strides.split(",")]:
        length = stride - 8
        n = int(a.gbytes * 1e9) // stride
        arena = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
        engine.gen_fixed(arena, stride, length, n, 0, w.seed, w.hdr)
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        run = lambda: engine.checksum_fixed(arena, stride, length, n, pseudo, N_FLOWS, out=out)  # noqa: E731
        ref, res, kern = None, {k: [] for k in arms}, {}
        for r in range(a.rounds):
            for name in (list(arms) if r % 2 == 0 else list(arms)[::-1]):
                engine.tune(**arms[name])
                try:
                    res[name].append(timed(run, a.iters))
                    kern[name] = last_kernel()
                    if ref is None:
                        ref = out.clone()
                    assert torch.equal(out, ref), (stride, name)
                finally:
                    engine.tune()
        for name, v in res.items():
            ms = statistics.median(v)
            print(json.dumps({"stride": stride, "length": length, "packets": n, "arm": name, "kernel": kern[name],
                              "ms": round(ms, 4), "rounds_ms": [round(x, 4) for x in v],
                              "frac_of_8TBs": round(n * (length + 2) / (ms / 1e3) / 8e12, 4)}), flush=True)
        del arena, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

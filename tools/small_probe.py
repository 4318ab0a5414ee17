#!/usr/bin/env python3
"""cfg1-shape probe: checksum vs RX-verify (2-B vs 1-B results per packet) and
the same bytes as 1 KiB packets, to separate the result stores and the packet
count from the read stream.  Median HIP-event kernel ms.

    python tools/small_probe.py [--mi 256]
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


def timed(fn, iters=10):
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
    ap.add_argument("--mi", type=int, default=256)
    a = ap.parse_args()
    engine.require_gpu()
    n = a.mi << 20
    arena = torch.empty(n * 24, dtype=torch.uint8, device="cuda")
    engine.gen_fixed(arena, 24, 20, n, 0, 1, 0)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    big_n = n * 24 // 1024
    cases = {
        "cfg1_checksum": lambda: engine.checksum_fixed(arena, 24, 20, n, out=out),
        "cfg1_verify": lambda: engine.verify_fixed(arena, 24, 20, n, ok=ok),
        "same_bytes_1KiB_pkts": lambda: engine.checksum_fixed(arena, 1024, 1024, big_n, out=out),
    }
    for name, fn in cases.items():
        for arm, kw in {"default": {}, "small": {"flat_tiny": False}}.items():
            if name.startswith("same") and arm == "small":
                continue
            engine.tune(**kw)
            ms = statistics.median(timed(fn) for _ in range(3))
            print(json.dumps({"case": name, "arm": arm, "packets": big_n if name.startswith("same") else n,
                              "ms": round(ms, 4), "read_GBps": round(n * 24 / ms / 1e6, 1)}), flush=True)
    engine.tune()


if __name__ == "__main__":
    main()

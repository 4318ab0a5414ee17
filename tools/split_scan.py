#!/usr/bin/env python3
"""Does a 75 GB cfg5 batch run slower because of the allocation or the launch?

Arms (all over the same 8M packets, interleaved in one process):
  one      one allocation, one launch over all 8M packets
  slices4  one allocation, 4 launches over contiguous 2M-packet slices
  slices8  one allocation, 8 launches over 1M-packet slices
  allocs4  4 separate allocations of 2M packets, 4 launches
"""
from __future__ import annotations

import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from pip_amd import engine  # noqa: E402
from pip_amd.workloads import CFG5, N_FLOWS  # noqa: E402


def timed(fn, iters=8):
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
    engine.require_gpu()
    w, n = CFG5, 8 << 20
    _, pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)
    arena = torch.empty(n * w.stride, dtype=torch.uint8, device="cuda")
    engine.gen_fixed(arena, w.stride, w.length, n, 0, w.seed, w.hdr)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    parts = []
    for k in range(4):
        p = torch.empty((n // 4) * w.stride, dtype=torch.uint8, device="cuda")
        engine.gen_fixed(p, w.stride, w.length, n // 4, k * (n // 4), w.seed, w.hdr)
        parts.append(p)

    def sliced(k):
        m = n // k

        def run():
            for j in range(k):
                engine.checksum_fixed(arena[j * m * w.stride:(j + 1) * m * w.stride], w.stride, w.length, m, pseudo,
                                      N_FLOWS, None, j * m, out=out[j * m:(j + 1) * m])
        return run

    def allocs():
        m = n // 4
        for j in range(4):
            engine.checksum_fixed(parts[j], w.stride, w.length, m, pseudo, N_FLOWS, None, j * m,
                                  out=out[j * m:(j + 1) * m])

    arms = {"one": sliced(1), "slices4": sliced(4), "slices8": sliced(8), "allocs4": allocs}
    ref = engine.checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS).clone()
    res = {}
    for _ in range(3):
        for name, fn in arms.items():
            res.setdefault(name, []).append(timed(fn))
            assert torch.equal(out, ref), name
    nbytes = (w.length + 2) * n
    for name, ms in res.items():
        m = statistics.median(ms)
        print(json.dumps({"arm": name, "ms": round(m, 4), "GBps": round(nbytes / m / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Does the flat kernel's small-batch rate depend on the allocation?  cfg2's
4M-packet batch (6.2 GB) timed in its own allocation and as a view at the
start / middle of a 75 GB allocation, arms interleaved.

    python tools/alloc_probe.py
"""
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


def main():
    engine.require_gpu()
    w, n = CFG2, 4 << 20
    nbytes = n * w.stride
    pseudo = engine.gen_flows(w.family, N_FLOWS, w.seed, w.proto)[1]
    own = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    big = torch.empty(12 * nbytes, dtype=torch.uint8, device="cuda")
    views = {"own": own, "big_start": big[:nbytes], "big_mid": big[6 * nbytes:7 * nbytes],
             "big_end": big[11 * nbytes:]}
    for v in views.values():
        engine.gen_fixed(v, w.stride, w.length, n, 0, w.seed, w.hdr)
    res = {}
    for _ in range(5):
        for k, v in views.items():
            res.setdefault(k, []).append(timed(lambda v=v: engine.checksum_fixed(v, w.stride, w.length, n, pseudo, N_FLOWS), 10))
    alg = (w.length + 2) * n
    for k, ms in res.items():
        m = statistics.median(ms)
        print(json.dumps({"arm": k, "ms": round(m, 4), "GBps": round(alg / m / 1e6, 1)}), flush=True)
    # per-launch spread inside one back-to-back sequence
    st = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(21)]
    ev[0].record(st)
    for i in range(20):
        engine.checksum_fixed(own, w.stride, w.length, n, pseudo, N_FLOWS)
        ev[i + 1].record(st)
    torch.cuda.synchronize()
    print(json.dumps({"per_launch_ms": [round(ev[i].elapsed_time(ev[i + 1]), 4) for i in range(20)]}))


if __name__ == "__main__":
    main()

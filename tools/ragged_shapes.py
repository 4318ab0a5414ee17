#!/usr/bin/env python3
"""Ragged kernel vs packet-length distribution, next to the fixed-stride path
on the same arena where one exists (uniform lengths give a packed arena whose
stride is roundup16(len), i.e. the fixed layout).

    python tools/ragged_shapes.py [--iters 10]

One JSON line per (shape, path): median kernel ms (HIP events), algorithmic GB/s.
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
from pip_amd.workloads import CFG4, N_FLOWS  # noqa: E402
from size_scan import timed  # noqa: E402

SHAPES = [("uniform_8980", 8980, 2 << 20), ("uniform_1480", 1480, 8 << 20), ("uniform_512", 512, 16 << 20),
          ("uniform_128", 128, 32 << 20), ("uniform_64", 64, 64 << 20), ("uniform_40", 40, 64 << 20),
          ("uniform_20", 20, 128 << 20), ("zipf_cfg4", 0, 8 << 20), ("zipf_cfg4_32M", 0, 32 << 20),
          ("zipf_plus192", -192, 8 << 20), ("zipf_plus448", -448, 8 << 20), ("zipf_plus960", -960, 8 << 20)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    engine.require_gpu()
    w = CFG4
    pseudo = engine.gen_flows(w.family, N_FLOWS, w.seed, w.proto)[1]
    for payload, n in ((1460, 8 << 20), (8960, 2 << 20)):
        # pip's TX chain shape: [20-B TCP header][payload] per packet, segments 16-B aligned
        name = f"chain_tcp_{payload}"
        if a.only and name not in a.only.split(","):
            continue
        slot = 32 + (payload + 15) // 16 * 16
        arena = torch.randint(0, 256, (n * slot,), dtype=torch.uint8, device="cuda")
        base = torch.arange(n, dtype=torch.int64, device="cuda") * slot
        segs = torch.empty((2 * n, 2), dtype=torch.int64, device="cuda")
        segs[0::2, 0], segs[1::2, 0] = base, base + 32
        segs[0::2, 1], segs[1::2, 1] = 20, payload  # len in the low u32, flow 0 in the high one
        seg_begin = torch.arange(0, 2 * n + 1, 2, dtype=torch.int64, device="cuda")
        pkt_flow = (torch.arange(n, dtype=torch.int64, device="cuda") % N_FLOWS).to(torch.int32)
        run = lambda: engine.checksum_chains(arena, segs, seg_begin, pkt_flow, pseudo)  # noqa: E731
        ms = statistics.median(timed(run, a.iters) for _ in range(5))
        nbytes = (20 + payload + 2) * n
        print(json.dumps({"shape": name, "packets": n, "gbytes": round(nbytes / 1e9, 2), "path": "chains",
                          "ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1)}), flush=True)
        del arena, segs, seg_begin, pkt_flow, base
        torch.cuda.empty_cache()
    for name, length, n in SHAPES:
        if a.only and name not in a.only.split(","):
            continue
        if length > 0:
            lengths = torch.full((n,), length, dtype=torch.int32, device="cuda")
        elif length < 0:  # cfg4's Zipf lengths shifted up by -length bytes (capped at 9000)
            z = torch.empty(n, dtype=torch.int32, device="cuda")
            engine.call("pipck_gen_zipf_lengths", engine._ptr(z), n, 0, w.seed, engine.current_stream())
            lengths = torch.clamp(z - length, max=9000)
        else:
            lengths = None
        arena, desc, lens = engine.gen_ragged(n, 0, w.seed, w.hdr, N_FLOWS, lengths=lengths)
        nbytes = int(lens.to(torch.int64).sum().item()) + 2 * n
        arms = {"ragged": lambda: engine.checksum_ragged(arena, desc, pseudo)}
        if 0 < length <= 49:  # tiny segments: lane-per-segment tiles vs the chunk stream
            def ragged_stream():
                engine.tune(tiny_tiles=False)
                try:
                    return engine.checksum_ragged(arena, desc, pseudo)
                finally:
                    engine.tune()
            arms["ragged_no_tiny"] = ragged_stream
        if length > 0:
            stride = (length + 15) // 16 * 16

            def fixed(**kw):
                engine.tune(**kw)
                try:
                    return engine.checksum_fixed(arena, stride, length, n, pseudo, N_FLOWS)
                finally:
                    engine.tune()
            arms["fixed"] = fixed
            if stride < 1024:  # short strides: the row-stream kernel vs the per-packet ones
                arms["fixed_no_flat_small"] = lambda: fixed(flat_small=False)
        res, ref = {}, None
        for _ in range(5):
            for k, fn in arms.items():
                res.setdefault(k, []).append(timed(fn, a.iters))
                out = fn()
                if ref is None:
                    ref = out.clone()
                elif k.startswith("fixed") or k == "ragged_no_tiny":
                    # fixed-path flows are (origin + i) % n_flows, the same as gen_ragged's descriptors
                    assert torch.equal(out, ref), name
        for k, ms in res.items():
            m = statistics.median(ms)
            print(json.dumps({"shape": name, "packets": n, "gbytes": round(nbytes / 1e9, 2), "path": k,
                              "ms": round(m, 4), "GBps": round(nbytes / m / 1e6, 1)}), flush=True)
        del arena, desc, lens
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

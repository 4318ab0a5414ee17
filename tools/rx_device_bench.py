#!/usr/bin/env python3
"""Rate of pipck_rx_verify_device: received IP packets already in HBM, byte-packed.

    python tools/rx_device_bench.py [--packets 8388608] [--iters 10] [--warm 40]

Synthetic frames built on the device: cfg4's Zipf L4 lengths (64-9,000 B, the
same generator), half TCP/IPv4, a quarter UDP/IPv4, a quarter TCP/IPv6, headers
well formed (versions, lengths, protocols) and every other byte random -- the
checksums do not verify, but each packet takes the full path (IPv4 header sum,
pseudo-header, payload verdict), which is what is timed; verdict parity is
tests/test_gpu_rx.py's job.  Reports, one JSON line each: pass 1 alone
(k_packedb over the frames, no pseudo-header: pipck_checksum_packed_bytes) and
the whole verifier (k_packedb<RX>: the same stream with each tile's headers
parsed and judged at its end), as frame bytes per second vs the 8 TB/s HBM
peak; algorithmic bytes = frame bytes read + the 2-B sum / 1-B verdict
written per packet.
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))


def build(n: int, seed: int):
    import torch

    from pip_amd import engine
    from pip_amd.workloads import CFG4

    g = torch.Generator(device="cuda").manual_seed(seed)
    l4 = torch.empty(n, dtype=torch.int32, device="cuda")
    engine.call("pipck_gen_zipf_lengths", engine._ptr(l4), n, 0, CFG4.seed, engine.current_stream())
    kind = torch.randint(0, 4, (n,), device="cuda", generator=g)  # 0,1 TCP/IPv4; 2 UDP/IPv4; 3 TCP/IPv6
    v6 = kind == 3
    hl = torch.where(v6, 40, 20).to(torch.int32)
    frame = l4 + hl
    lens = frame.to(torch.int16)
    tile_off = engine.packed_bytes_index(lens)
    total = int(tile_off[-1].item())
    arena = torch.randint(0, 256, ((total + 16 + 15) // 16 * 16,), dtype=torch.uint8, device="cuda", generator=g)
    starts = torch.cumsum(frame.to(torch.int64), 0) - frame.to(torch.int64)
    proto = torch.where(kind == 2, 17, 6)

    def put(col: int, val, mask=None):
        idx = starts + col
        if mask is not None:
            idx, val = idx[mask], (val[mask] if torch.is_tensor(val) else val)
        arena[idx] = (val if torch.is_tensor(val) else torch.full_like(idx, val)).to(torch.uint8)

    v4 = ~v6
    put(0, 0x45, v4)
    put(2, frame >> 8, v4)
    put(3, frame & 0xFF, v4)
    put(6, 0, v4)  # no fragment
    put(7, 0, v4)
    put(9, proto, v4)
    put(0, 0x60, v6)
    put(4, l4 >> 8, v6)
    put(5, l4 & 0xFF, v6)
    put(6, 6, v6)
    return arena, lens, tile_off, total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=8 << 20)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warm", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch

    from bench import last_kernel
    from pip_amd import engine
    from size_scan import timed_b2b

    engine.require_gpu()
    n = a.packets
    arena, lens, tile_off, total = build(n, 11)
    sums = torch.empty(n, dtype=torch.int16, device="cuda")
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    nbytes = arena.numel()

    def pass1():
        engine.call("pipck_checksum_packed_bytes_n", engine._ptr(arena), nbytes, engine._ptr(lens),
                    engine._ptr(tile_off), n, None, 0, None, 0, engine._ptr(sums), None, engine.current_stream())

    def full():
        engine.call("pipck_rx_verify_device", engine._ptr(arena), nbytes, engine._ptr(lens), engine._ptr(tile_off),
                    n, engine._ptr(ok), None, engine.current_stream())

    res = {"pass1": [], "rx_verify_device": []}
    kern = {}
    for rnd in range(a.rounds):
        for name, fn in (("pass1", pass1), ("rx_verify_device", full)) if rnd % 2 == 0 else \
                (("rx_verify_device", full), ("pass1", pass1)):
            for _ in range(a.warm):
                fn()
            res[name].append(timed_b2b(fn, a.iters))
            kern[name] = last_kernel().split("(")[0]
    v = ok.cpu().numpy()
    hist = {int(k): int(c) for k, c in zip(*__import__("numpy").unique(v, return_counts=True))}
    for name, ms in res.items():
        m = statistics.median(ms)
        algo = total + (n if name == "rx_verify_device" else 2 * n)
        print(json.dumps({"what": name, "packets": n, "frame_bytes": total, "last_kernel": kern[name], "ms": round(m, 4),
                          "rounds_ms": [round(x, 4) for x in ms], "GBps": round(algo / m / 1e6, 1),
                          "frac": round(algo / m / 1e6 / 8000, 4),
                          **({"verdicts": hist} if name == "rx_verify_device" else {})}), flush=True)


if __name__ == "__main__":
    main()

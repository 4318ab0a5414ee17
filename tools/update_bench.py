#!/usr/bin/env python3
"""RFC 1624 incremental update vs full recomputation, on the
device-resident cfg5 batch (8M x 8,980-B TCP/IPv4 segments, 75 GB).

    python tools/update_bench.py [--packets 8388608]

Arms, each timed with HIP events (median of 10 launches):
  recompute   pipck_checksum_fixed over every byte (what pip does after any edit)
  ports       rewrite the 4 port bytes of every packet, patch th_sum
  seq_ack     rewrite the 8 sequence/ack bytes, patch th_sum
  nat         ports + a new flow table (addresses behind the pseudo-header)
After the timed launches the batch is re-checksummed and must verify (every
patched field makes its packet sum to 0xFFFF).  One JSON line per arm.
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
from pip_amd.workloads import CFG5, N_FLOWS  # noqa: E402


def timed(fn, iters=10):
    st = torch.cuda.current_stream()
    ms = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        fn()
        b.record(st)
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b))
    return statistics.median(ms)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=8 << 20)
    a = ap.parse_args()
    engine.require_gpu()
    w, n = CFG5, a.packets
    arena = torch.empty(n * w.stride, dtype=torch.uint8, device="cuda")
    engine.gen_fixed(arena, w.stride, w.length, n, 0, w.seed, w.hdr)
    _, pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)
    _, pseudo2 = engine.gen_flows(4, N_FLOWS, w.seed + 1, w.proto)
    # store pip's checksums into th_sum (offset 16) so the batch is consistent
    out = engine.checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS)
    field = arena.view(n, w.stride)[:, 16:18]
    field.copy_(out.view(torch.uint8).view(n, 2).flip(1))  # htons
    new4 = torch.randint(0, 256, (n * 4,), dtype=torch.uint8, device="cuda")
    new8 = torch.randint(0, 256, (n * 8,), dtype=torch.uint8, device="cuda")
    tables = [pseudo, pseudo2]
    nat_state = {"cur": 0}

    def nat():
        old, new = tables[nat_state["cur"]], tables[nat_state["cur"] ^ 1]
        engine.update_fixed(arena, w.stride, n, 0, w.length, 16, 0, 4, new4, 4, old, new, N_FLOWS)
        nat_state["cur"] ^= 1

    arms = {
        "recompute": lambda: engine.checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS, out=out),
        "ports": lambda: engine.update_fixed(arena, w.stride, n, 0, w.length, 16, 0, 4, new4, 4),
        "seq_ack": lambda: engine.update_fixed(arena, w.stride, n, 0, w.length, 16, 4, 8, new8, 8),
        "nat": nat,
    }
    res = {k: timed(fn) for k, fn in arms.items()}
    if nat_state["cur"]:  # leave the batch under the first flow table
        nat()
    ok = engine.verify_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS)
    assert bool(ok.all()), "patched batch does not verify"
    for k, ms in res.items():
        print(json.dumps({"tool": "update_bench", "arm": k, "packets": n, "ms": round(ms, 4),
                          "mpkt_per_s": round(n / ms / 1e3, 1),
                          "vs_recompute": round(res["recompute"] / ms, 1)}), flush=True)


if __name__ == "__main__":
    main()

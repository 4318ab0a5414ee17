#!/usr/bin/env python3
"""Why does cfg2's kernel time depend on the calling context?  One process,
one arena; both fixed-stride schedules timed back to back (bench.py's way)
with the result array (a) preallocated once after the arena, as bench.py does,
(b) allocated fresh by every call (size_scan.py), (c) preallocated BEFORE the
arena, (d) a view at a 4 KiB offset inside a bigger buffer.  Prints one JSON
line per (variant, schedule): median per-dispatch ms over rounds, and the
result array's address mod 2 MiB."""
from __future__ import annotations

import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parent))

import torch  # noqa: E402

from pip_amd import engine  # noqa: E402
from pip_amd.workloads import CFG2, N_FLOWS  # noqa: E402
from size_scan import timed_b2b  # noqa: E402


def main():
    engine.require_gpu()
    w, n = CFG2, CFG2.n_packets
    pre = torch.empty(n, dtype=torch.int16, device="cuda")  # (c): before the arena
    pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)[1]
    arena = torch.empty(n * w.stride, dtype=torch.uint8, device="cuda")
    engine.gen_fixed(arena, w.stride, w.length, n, 0, w.seed, w.hdr)
    post = torch.empty(n, dtype=torch.int16, device="cuda")  # (a): after, as bench.py
    big = torch.empty(n + 4096, dtype=torch.int16, device="cuda")
    shifted = big[2048:2048 + n]  # (d): 4 KiB into a bigger buffer
    variants = {"bench_post": post, "per_call": None, "pre_arena": pre, "shift_4k": shifted}
    scheds = {"k_flat_coop": {}, "k_flat": {"alt_flat_schedule": True}}
    res = {}
    for r in range(4):
        for vname, out in variants.items():
            for sname, kw in scheds.items():
                engine.tune(**kw)
                fn = (lambda: engine.checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS)) if out is None \
                    else (lambda o=out: engine.checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS, out=o))
                res.setdefault((vname, sname), []).append(timed_b2b(fn, 20))
                engine.tune()
    for (vname, sname), v in res.items():
        out = variants[vname]
        print(json.dumps({"variant": vname, "schedule": sname, "ms": round(statistics.median(v), 4),
                          "rounds": [round(x, 4) for x in v],
                          "out_addr_mod_2MiB": None if out is None else out.data_ptr() % (2 << 20),
                          "arena_addr_mod_2MiB": arena.data_ptr() % (2 << 20)}), flush=True)


if __name__ == "__main__":
    main()

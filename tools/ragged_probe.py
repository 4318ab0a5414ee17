#!/usr/bin/env python3
"""Ragged-kernel row-depth probe on cfg4 (8M and 32M packets), arms interleaved.

    python tools/ragged_probe.py

Arms set pipck_tune(0, loads, 0, flags) directly: loads = rows in flight
(3/5/9 pipelined), flags bit 4 = no packed-tile addressing.  The loads-only
numbers in profiles/r01_ragged_probe_loads_only.jsonl came from a temporary
build whose flags bit 6 compiled the reduce out (removed since).
"""
import sys, json, statistics
sys.path.insert(0, "/root/repo")
import torch
from pip_amd import engine, _lib
from pip_amd.workloads import CFG4, N_FLOWS
sys.path.insert(0, "/root/repo/tools")
from size_scan import timed
engine.require_gpu()
lib = _lib.load()
w = CFG4
pseudo = engine.gen_flows(w.family, N_FLOWS, w.seed, w.proto)[1]
for n in (8 << 20, 32 << 20):
    arena, desc, lens = engine.gen_ragged(n, 0, w.seed, w.hdr, N_FLOWS)
    nbytes = int(lens.to(torch.int64).sum().item()) + 2 * n
    run = lambda: engine.checksum_ragged(arena, desc, pseudo)
    arms = {"u4": (4, 0), "u8": (8, 0), "u16": (16, 0), "u2": (2, 0), "pipe4": (5, 0), "pipe2": (3, 0),
            "u4_unpacked": (4, 16)}
    res = {}
    for rnd in range(5):
        for k, (loads, fl) in arms.items():
            lib.pipck_tune(0, loads, 0, fl)
            res.setdefault(k, []).append(timed(run, 10))
    lib.pipck_tune(0, 0, 0, 0)
    for k, ms in res.items():
        m = statistics.median(ms)
        print(json.dumps({"packets": n, "arm": k, "ms": round(m, 4), "GBps": round(nbytes / m / 1e6, 1)}), flush=True)
    del arena, desc
    torch.cuda.empty_cache()

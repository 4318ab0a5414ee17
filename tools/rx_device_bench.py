#!/usr/bin/env python3
"""Rate of pipck_rx_verify_device: received IP packets already in HBM, byte-packed.

    python tools/rx_device_bench.py [--packets 8388608] [--iters 10] [--warm 40]

Synthetic frames built on the device (engine.gen_rx_frames): cfg4's Zipf L4
lengths (64-9,000 B, the same generator), half TCP/IPv4, a quarter UDP/IPv4, a
quarter TCP/IPv6, every other byte random, checksum fields filled in by the
engine's ragged kernel -- so the verdict histogram is all 7 (PIPCK_RX_VERIFIED)
but for UDP/IPv4 frames whose checksum came out 0 (3, unchecked).  Reports, one JSON line each: pass 1 alone
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


def traffic_ratio(tag: str, kernel: str, algo_bytes: int) -> dict:
    """PMC traffic of this kernel on this workload, per launch, from
    profiles/traffic_rx_<tag>.json (tools/pmc_rx.sh writes it with the library's
    sha256): {"traffic": bytes, "traffic_ratio": traffic / algorithmic bytes} when the
    file was measured on this kernel of this build, else {}."""
    import hashlib

    f = ROOT / "profiles" / f"traffic_rx_{tag}.json"
    if not f.exists():
        return {}
    t = json.loads(f.read_text())
    lib = ROOT / "pip_amd" / "lib" / "libpipck.so"
    sha = hashlib.sha256(lib.read_bytes()).hexdigest() if lib.exists() else None
    if t.get("lib_sha256") != sha or t.get("kernel", "").split("(")[0] != kernel.split("(")[0]:
        return {"traffic": None, "traffic_note": "traffic file from another build or kernel"}
    tb = t["hbm_bytes_per_launch"]
    return {"traffic": tb, "traffic_ratio": round(tb / algo_bytes, 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=8 << 20)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warm", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--rings", default="ring_sparse_9216,ring_dense_1536,ring_dense_9216,ring_short_2048,ring_short_1024")
    ap.add_argument("--tune", default="{}", help="engine.tune kwargs for the packed arms and the default (groups) ring arm, JSON")
    ap.add_argument("--skip-packed", action="store_true", help="rings only")
    ap.add_argument("--arms", default="groups,kring,rows,slots",
                    help="ring schedules to time; groups:NAME = the default with --tunes[NAME]")
    ap.add_argument("--tunes", default="{}", help='JSON {"NAME": engine.tune kwargs} for groups:NAME arms')
    a = ap.parse_args()
    tune_default = json.loads(a.tune)
    tunes = json.loads(a.tunes)
    import torch

    from bench import last_kernel
    from pip_amd import engine
    from size_scan import timed_b2b

    engine.require_gpu()
    n = a.packets
    if a.skip_packed:
        arena = lens = tile_off = None
        total = 0
    else:
        arena, lens, tile_off, _, _, _ = engine.gen_rx_frames(n, 11)
        total = int(tile_off[-1].item())
    sums = torch.empty(n, dtype=torch.int16, device="cuda")
    ok = torch.empty(n, dtype=torch.uint8, device="cuda")
    nbytes = arena.numel() if arena is not None else 0

    def pass1():
        engine.call("pipck_checksum_packed_bytes_n", engine._ptr(arena), nbytes, engine._ptr(lens),
                    engine._ptr(tile_off), n, None, 0, None, 0, engine._ptr(sums), None, engine.current_stream())

    def full():
        engine.call("pipck_rx_verify_device", engine._ptr(arena), nbytes, engine._ptr(lens), engine._ptr(tile_off),
                    n, engine._ptr(ok), None, engine.current_stream())

    res = {"pass1": [], "rx_verify_device": []}
    kern = {}
    engine.tune(**tune_default)
    for rnd in range(0 if a.skip_packed else a.rounds):
        for name, fn in (("pass1", pass1), ("rx_verify_device", full)) if rnd % 2 == 0 else \
                (("rx_verify_device", full), ("pass1", pass1)):
            for _ in range(a.warm):
                fn()
            res[name].append(timed_b2b(fn, a.iters))
            kern[name] = last_kernel().split("(")[0]
    engine.tune()
    # rings: frames in fixed-size slots (pipck_rx_verify_ring), sparse (the same
    # Zipf frames in 9,216-B slots), dense (1,480-B L4 in 1,536-B slots, 8,900-B
    # L4 in 9,216-B slots) and short frames in small slots (200-B L4 in 2 KiB,
    # 100-B L4 in 1 KiB)
    rings = (("ring_sparse_9216", 9216, 0, n), ("ring_dense_1536", 1536, 1480, n), ("ring_dense_9216", 9216, 8900, n // 2),
             ("ring_short_2048", 2048, 200, n), ("ring_short_1024", 1024, 100, n),
             # probes (not in the default set): every slot filled to the byte (IPv4 frames of 9,216 B;
             # IPv6 ones 20 B longer would not fit, so the L4 length leaves room for both)
             ("ring_full_9216", 9216, 9216 - 40, n // 2), ("ring_full_1536", 1536, 1536 - 40, n))
    for tag, stride, l4_len, m in [r for r in rings if r[0] in a.rings.split(",")]:  # --rings none: packed only
        del arena
        torch.cuda.empty_cache()
        ring, rlens, _ = engine.gen_rx_ring(m, 11, stride, l4_len=l4_len)
        rok = torch.empty(m, dtype=torch.uint8, device="cuda")
        fbytes = int((rlens.to(torch.int64) & 0xFFFF).sum().item())

        def rfn():
            engine.call("pipck_rx_verify_ring", engine._ptr(ring), stride, engine._ptr(rlens), m, engine._ptr(rok),
                        engine.current_stream())

        # the three schedules, rounds interleaved, verdicts equal: the default slot
        # groups (k_ring), the row stream (k_ring_rx, flag bit 28) and slot by slot
        # (k_ring_slots, the wave-per-packet arm)
        ts = {k: [] for k in a.arms.split(",")}
        got = {}
        for _ in range(a.rounds):
            for arm in ts:
                if arm == "slots":
                    engine.tune(lanes_per_packet=256)
                elif arm == "rows":
                    engine.tune(alt_flat_schedule=True)
                elif arm == "kring":  # k_ring at every fill (no feedback)
                    engine.tune(**{**tune_default, "ring_adapt": False})
                elif arm.startswith("groups:"):
                    engine.tune(**tunes[arm.split(":", 1)[1]])
                else:
                    engine.tune(**tune_default)
                for _ in range(a.warm):
                    rfn()
                ts[arm].append(timed_b2b(rfn, a.iters))
                got[arm] = (last_kernel().split("(")[0], rok.clone())
        engine.tune()
        arms = list(got)
        assert all(torch.equal(got[arms[0]][1], got[k][1]) for k in arms)
        for arm, tl in ts.items():
            mr = statistics.median(tl)
            h = {int(k): int(c) for k, c in zip(*__import__("numpy").unique(got[arm][1].cpu().numpy(), return_counts=True))}
            print(json.dumps({"what": tag, "schedule": arm, "packets": m, "frame_bytes": fbytes,
                              "slot_bytes": m * stride, "last_kernel": got[arm][0], "ms": round(mr, 4),
                              "rounds_ms": [round(x, 4) for x in tl], "GBps": round((fbytes + m) / mr / 1e6, 1),
                              "frac": round((fbytes + m) / mr / 1e6 / 8000, 4), "verdicts": h,
                              **traffic_ratio(tag, got[arm][0], fbytes + m),
                              "verdicts_equal_across_schedules": True}), flush=True)
        del ring
        arena = torch.empty(1, device="cuda")
    if a.skip_packed:
        return
    v = ok.cpu().numpy()
    hist = {int(k): int(c) for k, c in zip(*__import__("numpy").unique(v, return_counts=True))}
    for name, ms in res.items():
        m = statistics.median(ms)
        algo = total + (n if name == "rx_verify_device" else 2 * n)
        print(json.dumps({"what": name, "packets": n, "frame_bytes": total, "last_kernel": kern[name], "ms": round(m, 4),
                          "rounds_ms": [round(x, 4) for x in ms], "GBps": round(algo / m / 1e6, 1),
                          "frac": round(algo / m / 1e6 / 8000, 4), **traffic_ratio(name, kern[name], algo),
                          **({"verdicts": hist} if name == "rx_verify_device" else {})}), flush=True)


if __name__ == "__main__":
    main()

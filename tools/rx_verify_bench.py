#!/usr/bin/env python3
"""RX batch verification rate (pipck_rx_verify, the per-packet verifier behind the
drop-in's pip_checksum_amd_verify_packets) from host memory: N TCP/IPv4 packets of a given size,
heap (copied into the queue's staging) or pinned (pipck_host_alloc: read in
place), one call per batch.  One JSON line per (size, batch, memory).

    python tools/rx_verify_bench.py [--sizes 1500,9000] [--batches 1024,16384,65536]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import numpy as np  # noqa: E402

from pip_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1500,9000")
    ap.add_argument("--batches", default="1024,16384,65536")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--packed", action="store_true",
                    help="also time pipck_host_rx_verify_packed on the same frames (they lie back to back)")
    a = ap.parse_args()
    lib = _lib.load()
    # the per-packet verifier through its C ABI (pipck_rx_verify): the drop-in's
    # pip_checksum_amd_verify_packets now sends batches that lie back to back in
    # one buffer -- as here -- to pipck_host_rx_verify_packed instead
    rxq = C.c_void_p()
    assert lib.pipck_rxq_create(None, C.byref(rxq)) == 0

    def fn(ptrs, lens, n, ok_ptr):
        good = C.c_uint64()
        assert lib.pipck_rx_verify(rxq, ptrs, lens, n, ok_ptr, C.byref(good)) == 0
        return good.value

    rng = np.random.default_rng(3)
    for size in (int(x) for x in a.sizes.split(",")):
        for n in (int(x) for x in a.batches.split(",")):
            total = size * n
            for mem in ("heap", "pinned"):
                if mem == "pinned":
                    p = lib.pipck_host_alloc(total)
                    buf = np.ctypeslib.as_array((C.c_uint8 * total).from_address(p))
                else:
                    buf = np.empty(total, dtype=np.uint8)
                buf[:] = rng.integers(0, 256, total, dtype=np.uint8)
                pk = buf.reshape(n, size)
                pk[:, 0] = 0x45
                pk[:, 2] = size >> 8
                pk[:, 3] = size & 0xFF
                pk[:, 6] = 0x40  # DF, offset 0: not a fragment (a fragment's L4 is not checked)
                pk[:, 7] = 0
                pk[:, 9] = 6
                base = buf.ctypes.data
                ptrs = (C.c_void_p * n)(*[base + i * size for i in range(n)])
                lens = (C.c_uint32 * n)(*([size] * n))
                ok = np.zeros(n, dtype=np.uint8)
                fn(ptrs, lens, n, ok.ctypes.data)  # warm
                ts = []
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    fn(ptrs, lens, n, ok.ctypes.data)
                    ts.append(time.perf_counter() - t0)
                t = statistics.median(ts)
                print(json.dumps({"tool": "rx_verify_bench", "packet_bytes": size, "batch": n, "memory": mem,
                                  "ms_per_call": round(t * 1e3, 4), "gib_per_s": round(total / t / 2**30, 3),
                                  "mpkt_per_s": round(n / t / 1e6, 3), "verified": int((ok == 7).sum()),
                                  "l4_checked": int(((ok & 4) != 0).sum())}), flush=True)
                if a.packed:  # the same frames, back to back: one DMA stream per chunk, verdicts on the device
                    ctx = C.c_void_p()
                    assert lib.pipck_ctx_create(-1, C.byref(ctx)) == 0
                    l16 = np.full(n, size, dtype=np.uint16)
                    ok2 = np.zeros(n, dtype=np.uint8)
                    good = C.c_uint64()
                    hp = lib.pipck_host_rx_verify_packed
                    assert hp(ctx, base, l16.ctypes.data, n, ok2.ctypes.data, C.byref(good)) == 0  # warm
                    ts = []
                    for _ in range(a.reps):
                        t0 = time.perf_counter()
                        hp(ctx, base, l16.ctypes.data, n, ok2.ctypes.data, C.byref(good))
                        ts.append(time.perf_counter() - t0)
                    t2 = statistics.median(ts)
                    assert np.array_equal(ok, ok2)
                    print(json.dumps({"tool": "rx_verify_bench", "api": "pipck_host_rx_verify_packed",
                                      "packet_bytes": size, "batch": n, "memory": mem,
                                      "ms_per_call": round(t2 * 1e3, 4), "gib_per_s": round(total / t2 / 2**30, 3),
                                      "mpkt_per_s": round(n / t2 / 1e6, 3), "verified": int(good.value),
                                      "verdicts_equal_drop_in": True}), flush=True)
                    lib.pipck_ctx_destroy(ctx)
                del pk, buf
                if mem == "pinned":
                    lib.pipck_host_free(C.c_void_p(p))


if __name__ == "__main__":
    main()

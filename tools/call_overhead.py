"""MEASUREMENT ONLY: host cost per call of the cfg1 bench step (1M IPv4
headers, launch-bound) -- the engine wrapper, a pre-bound ctypes call of the
same C ABI entry, and each with the per-dispatch event pair bench.py records.
One JSON line per arm: wall us per call over 2,000 back-to-back calls."""
import ctypes as C
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from pip_amd import _lib, engine
from pip_amd.workloads import CFG1, N_FLOWS


def main():
    engine.require_gpu()
    w, n = CFG1, 1 << 20
    arena = torch.empty(n * w.stride, dtype=torch.uint8, device="cuda")
    engine.gen_fixed(arena, w.stride, w.length, n, 0, w.seed, w.hdr)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    lib = _lib.load()
    fn = lib.pipck_checksum_fixed
    args = (C.c_void_p(arena.data_ptr()), w.stride, w.length, n, None, N_FLOWS, None, 0, C.c_void_p(out.data_ptr()),
            engine.current_stream())

    def wrapper():
        engine.checksum_fixed(arena, w.stride, w.length, n, None, N_FLOWS, None, 0, out=out)

    def bound():
        rc = fn(*args)
        if rc:
            _lib.check("pipck_checksum_fixed", rc)

    e0 = [torch.cuda.Event(enable_timing=True) for _ in range(2000)]
    e1 = [torch.cuda.Event(enable_timing=True) for _ in range(2000)]
    hip = C.CDLL("libamdhip64.so")
    hip.hipEventRecord.argtypes = [C.c_void_p, C.c_void_p]
    hip.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
    h0, h1 = [C.c_void_p() for _ in range(2000)], [C.c_void_p() for _ in range(2000)]
    for e in h0 + h1:
        assert hip.hipEventCreate(C.byref(e)) == 0
    stream = engine.current_stream()
    rec = hip.hipEventRecord
    for name, f, ev in (("wrapper", wrapper, None), ("bound", bound, None), ("wrapper+events", wrapper, "torch"),
                        ("bound+events", bound, "torch"), ("wrapper+hip_events", wrapper, "hip"),
                        ("bound+hip_events", bound, "hip")):
        for _ in range(200):
            f()
        torch.cuda.synchronize()
        t0 = time.perf_counter_ns()
        for i in range(2000):
            if ev == "torch":
                e0[i].record()
            elif ev == "hip":
                rec(h0[i], stream)
            f()
            if ev == "torch":
                e1[i].record()
            elif ev == "hip":
                rec(h1[i], stream)
        torch.cuda.synchronize()
        us = (time.perf_counter_ns() - t0) / 2000 / 1e3
        line = {"arm": name, "us_per_call": round(us, 2)}
        if ev == "torch":
            d = sorted(a.elapsed_time(b) * 1e3 for a, b in zip(e0, e1))
            line["event_pair_median_us"] = round(d[len(d) // 2], 2)
        elif ev == "hip":
            d = []
            for a, b in zip(h0, h1):
                ms = C.c_float()
                assert hip.hipEventElapsedTime(C.byref(ms), a, b) == 0
                d.append(ms.value * 1e3)
            d.sort()
            line["event_pair_median_us"] = round(d[len(d) // 2], 2)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()

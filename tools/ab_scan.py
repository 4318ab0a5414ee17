#!/usr/bin/env python3
"""Same-process A/B of libpipck builds (box-to-box variation is a few %,
larger than most kernel changes).

    python tools/ab_scan.py [--only cfg2,cfg4] pip_amd/lib/ab/libpipck_base.so [more.so ...]

Each given library is an arm named after its file stem (minus "libpipck_"),
arm "cur" = pip_amd/lib/libpipck.so; all run the same device batches
(generated once), rounds interleaved, results checked equal.  One JSON line
per (workload, arm).
"""
from __future__ import annotations

import ctypes as C
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from pip_amd import _lib, engine  # noqa: E402
from pip_amd.workloads import CFG2, CFG3, CFG4, CFG5, N_FLOWS  # noqa: E402
from size_scan import timed  # noqa: E402


def bind(lib):
    for name in ("pipck_checksum_fixed", "pipck_checksum_ragged"):
        res, args = _lib.SIGNATURES[name]
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    return lib


def main():
    engine.require_gpu()
    args = sys.argv[1:]
    only = None
    if args and args[0] == "--only":
        only, args = set(args[1].split(",")), args[2:]
    libs = {Path(a).stem.replace("libpipck_", ""): bind(C.CDLL(str(Path(a).resolve()))) for a in args}
    libs["cur"] = bind(_lib.load())
    p = engine._ptr
    for w, n in ((CFG2, 4 << 20), (CFG3, 1 << 20), (CFG5, 8 << 20), (CFG4, 8 << 20)):
        if only and f"cfg{w.cfg}" not in only:
            continue
        pseudo = engine.gen_flows(w.family, N_FLOWS, w.seed, w.proto)[1]
        out = torch.empty(n, dtype=torch.int16, device="cuda")
        st = engine.current_stream()
        if w.ragged:
            arena, desc, lens = engine.gen_ragged(n, 0, w.seed, w.hdr, N_FLOWS)
            nbytes = int(lens.to(torch.int64).sum().item()) + 2 * n
            runs = {k: (lambda lib=lib: lib.pipck_checksum_ragged(p(arena), p(desc), n, p(pseudo), p(out), None, st))
                    for k, lib in libs.items()}
        else:
            arena = torch.empty(n * w.stride, dtype=torch.uint8, device="cuda")
            engine.gen_fixed(arena, w.stride, w.length, n, 0, w.seed, w.hdr)
            nbytes = (w.length + 2) * n
            runs = {k: (lambda lib=lib: lib.pipck_checksum_fixed(p(arena), w.stride, w.length, n, p(pseudo),
                                                                 N_FLOWS, None, 0, p(out), st))
                    for k, lib in libs.items()}
        res, ref = {}, None
        for _ in range(7):
            for k, fn in runs.items():
                res.setdefault(k, []).append(timed(fn, 10))
                out.zero_()
                assert fn() == 0
                if ref is None:
                    ref = out.clone()
                assert torch.equal(out, ref), k
        for k, ms in res.items():
            m = statistics.median(ms)
            print(json.dumps({"workload": w.name, "packets": n, "arm": k, "ms": round(m, 4),
                              "GBps": round(nbytes / m / 1e6, 1)}), flush=True)
        del arena
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

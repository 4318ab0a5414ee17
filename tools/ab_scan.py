#!/usr/bin/env python3
"""A/B of libpipck builds on one GPU box (box-to-box variation is a few %,
larger than most kernel changes).

    python tools/ab_scan.py [--only cfg2,cfg4] [--rounds 3] pip_amd/lib/ab/libpipck_base.so [more.so ...] [cur@1024]

Each given library is an arm named after its file stem (minus "libpipck_"),
arm "cur" = pip_amd/lib/libpipck.so.  Every (round, arm) runs in its OWN
process (PIPCK_LIB selects the build): two builds loaded into one process
share kernel symbol names, and the HIP runtime then launches one build's
kernels for both.  Rounds alternate the arms; each process generates the same
device batches and reports the median kernel time; the results' hashes must
agree across arms.  One JSON line per (workload, arm): median over rounds.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import statistics
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
WORKLOADS = {"cfg1": 256 << 20, "cfg1p": 256 << 20, "cfg2": 4 << 20, "cfg3": 1 << 20, "cfg5": 8 << 20, "cfg4": 8 << 20,
             "cfg4d": 8 << 20, "cfg4b": 8 << 20}


def worker(only: list[str], iters: int, warm: int = 0, b2b: bool = False) -> None:
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "tools"))
    import torch

    from pip_amd import engine
    from pip_amd.workloads import BY_CFG, N_FLOWS
    from size_scan import timed, timed_b2b

    engine.require_gpu()
    # placement probe: PIPCK_AB_PAD_MB of device memory held before the batches
    # are allocated, so the same build's arena lands elsewhere in HBM
    pad = torch.empty(int(os.environ.get("PIPCK_AB_PAD_MB", "0")) << 20, dtype=torch.uint8, device="cuda")
    for name in only:
        w, n = BY_CFG[int(name[3:4])], WORKLOADS[name]
        fam = w.family or (4 if name.endswith("p") else 0)  # cfg1p: cfg1 with IPv4 pseudo-headers
        pseudo = engine.gen_flows(fam, N_FLOWS, w.seed, w.proto or 6)[1] if fam else None
        if name == "cfg4b":  # cfg4 byte-packed: the layout bench.py runs (k_packedb)
            arena, lens16, tile_off, lens = engine.gen_packed_bytes(n, 0, w.seed, w.hdr)
            nbytes = int(lens.to(torch.int64).sum().item()) + 2 * n
            out = torch.empty(n, dtype=torch.int16, device="cuda")

            def run():  # the plain entry point: present in every build under A/B
                engine.call("pipck_checksum_packed_bytes", engine._ptr(arena), engine._ptr(lens16),
                            engine._ptr(tile_off), n, engine._ptr(pseudo), N_FLOWS, None, 0, engine._ptr(out),
                            engine.current_stream())
                return out
        elif w.ragged and not name.endswith("d"):  # cfg4: the 16-byte packed layout (k_packed)
            arena, lens16, tile_chunk, lens = engine.gen_packed(n, 0, w.seed, w.hdr)
            nbytes = int(lens.to(torch.int64).sum().item()) + 2 * n
            out = torch.empty(n, dtype=torch.int16, device="cuda")

            def run():  # the plain entry point: present in every build under A/B
                engine.call("pipck_checksum_packed", engine._ptr(arena), engine._ptr(lens16), engine._ptr(tile_chunk),
                            n, engine._ptr(pseudo), N_FLOWS, None, 0, engine._ptr(out), engine.current_stream())
                return out
        elif w.ragged:  # cfg4d: 16-byte descriptors (pipck_checksum_ragged)
            arena, desc, lens = engine.gen_ragged(n, 0, w.seed, w.hdr, N_FLOWS)
            nbytes = int(lens.to(torch.int64).sum().item()) + 2 * n
            run = lambda: engine.checksum_ragged(arena, desc, pseudo)  # noqa: E731
        else:
            arena = torch.empty(n * w.stride, dtype=torch.uint8, device="cuda")
            engine.gen_fixed(arena, w.stride, w.length, n, 0, w.seed, w.hdr)
            nbytes = (w.length + 2) * n
            out = torch.empty(n, dtype=torch.int16, device="cuda")

            def run():  # the plain entry point: present in every build under A/B
                engine.call("pipck_checksum_fixed", engine._ptr(arena), w.stride, w.length, n, engine._ptr(pseudo),
                            N_FLOWS, None, 0, engine._ptr(out), engine.current_stream())
                return out
        for _ in range(warm):  # past the GPU's post-idle clock ramp (DESIGN §5 "Warm-up")
            run()
        ms = statistics.median((timed_b2b if b2b else timed)(run, iters) for _ in range(3))
        digest = hashlib.sha256(run().cpu().numpy().tobytes()).hexdigest()[:16]
        tag = ("+pseudo" if fam and not w.family else "") + ("+desc" if name == "cfg4d" else "") + \
            ("+bytes" if name == "cfg4b" else "")
        print(json.dumps({"workload": w.name + tag, "packets": n, "ms": ms,
                          "bytes": nbytes, "sha": digest}), flush=True)
        del arena
        torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="cfg2,cfg3,cfg5,cfg4")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warm", type=int, default=0, help="untimed launches per workload before timing (clock ramp: 40)")
    ap.add_argument("--b2b", action="store_true", help="launches back to back as bench.py times them")
    ap.add_argument("--worker", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("libs", nargs="*")
    a = ap.parse_args()
    only = [x for x in a.only.split(",") if x]
    if a.worker:
        worker(only, a.iters, a.warm, a.b2b)
        return
    # an arm is a library path, or "path@MB" / "cur@MB": that build with MB of
    # device memory allocated before its batches (a placement probe)
    arms = {}
    for x in a.libs:
        lib, _, pad = x.partition("@")
        path = ROOT / "pip_amd" / "lib" / "libpipck.so" if lib == "cur" else Path(lib).resolve()
        name = "cur" if lib == "cur" else Path(lib).stem.replace("libpipck_", "")
        arms[name + (f"_pad{pad}" if pad else "")] = (str(path), pad or "0")
    arms.setdefault("cur", (str(ROOT / "pip_amd" / "lib" / "libpipck.so"), "0"))
    res: dict[tuple[str, str], list[float]] = {}
    meta: dict[str, dict] = {}
    for rnd in range(a.rounds):
        order = list(arms.items()) if rnd % 2 == 0 else list(reversed(arms.items()))
        for arm, (path, pad) in order:
            env = dict(os.environ, PIPCK_LIB=path, PIPCK_AB_PAD_MB=pad)
            r = subprocess.run([sys.executable, __file__, "--worker", "--only", ",".join(only), "--iters",
                                str(a.iters), "--warm", str(a.warm)] + (["--b2b"] if a.b2b else []), env=env, capture_output=True, text=True, timeout=600)
            if r.returncode:
                sys.stderr.write(r.stderr[-3000:])
                raise SystemExit(f"arm {arm} failed (rc {r.returncode})")
            for line in r.stdout.splitlines():
                if not line.startswith("{"):
                    continue
                d = json.loads(line)
                res.setdefault((d["workload"], arm), []).append(d["ms"])
                m = meta.setdefault(d["workload"], {"bytes": d["bytes"], "packets": d["packets"], "sha": d["sha"]})
                if m["sha"] != d["sha"]:
                    raise SystemExit(f"{d['workload']}: arm {arm} results differ from the first arm's")
    for (wl, arm), ms in res.items():
        m = statistics.median(ms)
        print(json.dumps({"workload": wl, "packets": meta[wl]["packets"], "arm": arm, "ms": round(m, 4),
                          "GBps": round(meta[wl]["bytes"] / m / 1e6, 1), "rounds": len(ms),
                          "rounds_ms": [round(x, 4) for x in ms]}), flush=True)


if __name__ == "__main__":
    main()

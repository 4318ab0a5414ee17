"""MEASUREMENT: the result array in HBM (bench.py's layout) against the same
kernel writing its 2-B results straight into pinned host memory (the place
pip needs them), on cfg2 / cfg4 / cfg5 -- the batch stays in HBM either way.
Arms interleaved per round, per-dispatch raw HIP event pairs (median of 20
after 40 warm-up launches), results compared.  One JSON line per (round,
workload, arm)."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from bench import HipEvents, last_kernel  # noqa: E402
from pip_amd import engine  # noqa: E402
from pip_amd.workloads import BY_CFG, N_FLOWS  # noqa: E402


def main():
    engine.require_gpu()
    for cfg in (2, 4, 5):
        w = BY_CFG[cfg]
        n = w.n_packets if cfg != 5 else 8 << 20
        pseudo = engine.gen_flows(w.family, N_FLOWS, w.seed, w.proto)[1]
        if w.ragged:
            arena, lens16, tile_off, _ = engine.gen_packed_bytes(n, 0, w.seed, w.hdr)

            def prep(out):
                return engine.prepare_checksum_packed_bytes(arena, lens16, tile_off, n, pseudo, N_FLOWS, None, 0,
                                                            out=out)[0]
        else:
            arena = torch.empty(n * w.stride, dtype=torch.uint8, device="cuda")
            engine.gen_fixed(arena, w.stride, w.length, n, 0, w.seed, w.hdr)

            def prep(out):
                return engine.prepare_checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS, None, 0,
                                                     out=out)[0]
        outs = {"hbm": torch.empty(n, dtype=torch.int16, device="cuda"),
                "pinned_host": torch.empty(n, dtype=torch.int16, pin_memory=True)}
        runs = {k: prep(o) for k, o in outs.items()}
        for rnd in range(3):
            for arm, run in runs.items():
                for _ in range(40):
                    run()
                ev = HipEvents(40, engine.current_stream().value)
                for i in range(20):
                    ev.record(2 * i)
                    run()
                    ev.record(2 * i + 1)
                torch.cuda.synchronize()
                d = sorted(ev.elapsed_s(2 * i, 2 * i + 1) for i in range(20))
                ev.destroy()
                print(json.dumps({"round": rnd, "workload": w.name, "arm": arm, "kernel_ms": round(d[10] * 1e3, 4),
                                  "last_kernel": last_kernel().split("(")[0]}), flush=True)
        torch.cuda.synchronize()
        assert torch.equal(outs["hbm"].cpu(), outs["pinned_host"]), w.name
        del arena, outs, runs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

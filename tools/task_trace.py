#!/usr/bin/env python3
"""Per-task timeline of the streaming kernels (internal trace, pipck_trace_tasks).

    python tools/task_trace.py [--only cfg2,cfg4,cfg5] [--arms '{"a": {...}}'] [--dump DIR]

For each workload (bench.py's layout: fixed strides -> k_flat, cfg4 -> the
packed kernel) and arm (engine.tune kwargs), the kernel runs a few untraced
launches, then one traced launch.  Every wave task stores {task, t_start,
t_end, XCC/HW id} on the 100 MHz wall clock.  Printed per launch (one JSON
line): span vs HIP-event time; the launch ramp (time until 99 % of the
resident wave slots hold a task) and the tail (time from the last task start
to the kernel end, and the mean number of busy slots over it); task
durations (median, p10, p90; first generation vs the rest); the idle gap
between consecutive tasks of one wave slot; per-XCD finish spread.
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pip_amd import engine  # noqa: E402
from pip_amd.workloads import BY_CFG, N_FLOWS  # noqa: E402

CLK = 100e6  # s_memrealtime


def analyse(rec: np.ndarray, ev_ms: float) -> dict:
    rec = rec[rec[:, 2] > 0]
    t0, t1 = rec[:, 1].astype(np.int64), rec[:, 2].astype(np.int64)
    base = t0.min()
    t0, t1 = t0 - base, t1 - base
    span = t1.max()
    dur = t1 - t0
    hw = rec[:, 3]
    xcc = (hw >> 32).astype(np.int64)
    # wave slot = XCC + (HW_ID: wave, simd, cu, sh, se); tasks of one slot in start order
    slot = hw & 0xFFFFFFFF
    key = xcc * (1 << 32) + slot.astype(np.int64)
    order = np.lexsort((t0, key))
    k_s, t0_s, t1_s = key[order], t0[order], t1[order]
    same = k_s[1:] == k_s[:-1]
    gaps = (t0_s[1:] - t1_s[:-1])[same]
    n_slots = len(np.unique(key))
    # busy slots over time (1 us bins)
    nb = int(span // 100) + 1
    busy = np.zeros(nb + 1)
    np.add.at(busy, (t0 // 100).astype(np.int64), 1)
    np.add.at(busy, (t1 // 100).astype(np.int64), -1)
    busy = np.cumsum(busy)[:nb]
    full = np.nonzero(busy >= 0.99 * n_slots)[0]
    ramp_us = float(full[0]) if len(full) else None
    last_start = t0.max()
    tail_busy = float(busy[int(last_start // 100):].mean()) if nb > last_start // 100 else None
    first_gen = t0 < np.sort(t0)[min(len(t0) - 1, n_slots)]
    xend = [int(t1[xcc == x].max()) for x in np.unique(xcc)]
    return {
        "tasks": int(len(rec)), "slots": int(n_slots), "event_ms": round(ev_ms, 4),
        "span_ms": round(span / CLK * 1e3, 4),
        "task_us": {"median": round(float(np.median(dur)) / 100, 2), "p10": round(float(np.percentile(dur, 10)) / 100, 2),
                    "p90": round(float(np.percentile(dur, 90)) / 100, 2),
                    "first_gen_median": round(float(np.median(dur[first_gen])) / 100, 2),
                    "later_median": round(float(np.median(dur[~first_gen])) / 100, 2) if (~first_gen).any() else None},
        "slot_gap_us": {"median": round(float(np.median(gaps)) / 100, 3) if len(gaps) else None,
                        "p90": round(float(np.percentile(gaps, 90)) / 100, 3) if len(gaps) else None,
                        "sum_over_slots_us": round(float(gaps.sum()) / 100 / max(n_slots, 1), 2)},
        "ramp_us_to_99pct_slots": ramp_us,
        "tail_us": round(float(span - last_start) / 100, 2), "tail_mean_busy_slots": round(tail_busy, 1) if tail_busy else None,
        "busy_slots_mean": round(float(busy.mean()), 1),
        "xcd_end_spread_us": round((max(xend) - min(xend)) / 100, 2), "xcds": len(xend),
        "first_task_end_us": round(float(t1.min()) / 100, 2),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="cfg2,cfg4,cfg5")
    ap.add_argument("--arms", default='{"default": {}}')
    ap.add_argument("--packets", type=int, default=0)
    ap.add_argument("--dump", default="")
    a = ap.parse_args()
    engine.require_gpu()
    lib = engine.load()
    arms = json.loads(a.arms)
    for c in [int(x.strip().lstrip("cfg")) for x in a.only.split(",")]:
        w = BY_CFG[c]
        n = a.packets or (8 << 20 if c == 5 else w.n_packets)
        pseudo = engine.gen_flows(w.family, N_FLOWS, w.seed, w.proto)[1] if w.family else None
        if w.ragged:
            arena, lens16, tile_chunk, lens = engine.gen_packed(n, 0, w.seed, w.hdr)
            run = lambda: engine.checksum_packed(arena, lens16, tile_chunk, n, pseudo, N_FLOWS)  # noqa: E731
        else:
            arena = torch.empty(n * w.stride, dtype=torch.uint8, device="cuda")
            engine.gen_fixed(arena, w.stride, w.length, n, 0, w.seed, w.hdr)
            run = lambda: engine.checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS)  # noqa: E731
        cap = n  # >= tasks for any arm (a task holds >= 1 packet)
        buf = torch.zeros(cap * 4, dtype=torch.int64, device="cuda")
        for name, kw in arms.items():
            engine.tune(**kw)
            ref = run().clone()
            for _ in range(3):
                run()
            engine.tune(**kw, trace=True)
            buf.zero_()
            engine.call("pipck_trace_tasks", engine._ptr(buf), cap)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = run()
            e1.record()
            torch.cuda.synchronize()
            engine.call("pipck_trace_tasks", None, 0)
            engine.tune()
            assert torch.equal(out, ref)
            rec = buf.view(-1, 4).cpu().numpy().view(np.uint64)
            used = rec[rec[:, 2] > 0]
            res = {"workload": w.name, "packets": n, "arm": name, **analyse(used, e0.elapsed_time(e1))}
            print(json.dumps(res), flush=True)
            if a.dump:
                Path(a.dump).mkdir(parents=True, exist_ok=True)
                np.save(Path(a.dump) / f"{w.name}_{name}.npy", used)
        del arena
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

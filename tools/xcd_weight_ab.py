#!/usr/bin/env python3
"""cfg2 under the XCD-weighted static deal (k_flat_xw) vs k_flat -- VERDICT r03 item 7.

    python tools/xcd_weight_ab.py [--packets N] [--rounds R] [--iters K] [--period M]

1. A traced launch of k_flat (pipck_trace_tasks) gives each XCD's mean task
   time on THIS box and batch; XCD x then keeps m_x = round(M * r_x / max r)
   of every M blocks dealt to it (r_x = 1 / mean task time), so faster XCDs
   take proportionally more of the tasks (pipck_tune_xcd_weights).
2. Traced launches of both arms: per-XCD finish times (the imbalance the deal
   is meant to remove).
3. Timed A/B in one process, arms interleaved round by round: the median of K
   per-launch HIP event pairs per arm and round; results checked equal.
One JSON line per step; the summary line last.  k_flat is cfg2's
other schedule since round 4 (the default is k_flat_coop), so both arms run
with tune bit 28 (alt_flat_schedule) set.
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
from pip_amd.workloads import CFG2, N_FLOWS  # noqa: E402


def last_kernel() -> str:
    import ctypes as C

    buf = C.create_string_buffer(4096)
    engine.load().pipck_last_launch(buf, len(buf))
    return buf.value.decode()


BASE = {"alt_flat_schedule": True}  # k_flat (and k_flat_xw), not k_flat_coop


def traced(run, cap):
    buf = torch.zeros(cap * 4, dtype=torch.int64, device="cuda")
    engine.tune(**BASE, trace=True)
    engine.call("pipck_trace_tasks", engine._ptr(buf), cap)
    torch.cuda.synchronize()
    out = run()
    torch.cuda.synchronize()
    engine.call("pipck_trace_tasks", None, 0)
    engine.tune(**BASE)
    rec = buf.view(-1, 4).cpu().numpy().view(np.uint64)
    rec = rec[rec[:, 2] > 0]
    t0 = rec[:, 1].astype(np.int64)
    t1 = rec[:, 2].astype(np.int64)
    base = t0.min()
    xcc = (rec[:, 3] >> 32).astype(np.int64)
    per = {}
    for x in range(8):
        sel = xcc == x
        per[x] = {"tasks": int(sel.sum()), "mean_task_us": float((t1[sel] - t0[sel]).mean()) / 100 if sel.any() else 0.0,
                  "end_us": float(t1[sel].max() - base) / 100 if sel.any() else 0.0}
    return out, per


def timed(run, iters):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for s, e in ev:
        s.record()
        run()
        e.record()
    torch.cuda.synchronize()
    return statistics.median(s.elapsed_time(e) for s, e in ev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=CFG2.n_packets)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--period", type=int, default=64)
    a = ap.parse_args()
    engine.require_gpu()
    engine.tune(**BASE)
    w, n = CFG2, a.packets
    pseudo = engine.gen_flows(4, N_FLOWS, w.seed, w.proto)[1]
    arena = torch.empty(n * w.stride, dtype=torch.uint8, device="cuda")
    engine.gen_fixed(arena, w.stride, w.length, n, 0, w.seed, w.hdr)
    out = torch.empty(n, dtype=torch.int16, device="cuda")
    run = lambda: engine.checksum_fixed(arena, w.stride, w.length, n, pseudo, N_FLOWS, out=out)  # noqa: E731
    for _ in range(5):
        run()
    ref = run().clone()
    k_default = last_kernel()
    _, per = traced(run, n)
    rate = {x: 1.0 / p["mean_task_us"] for x, p in per.items() if p["mean_task_us"] > 0}
    top = max(rate.values())
    m = [max(1, round(a.period * rate.get(x, top) / top)) for x in range(8)]
    print(json.dumps({"step": "calibrate", "packets": n, "kernel": k_default, "per_xcd": per, "weights": m,
                      "period": a.period}), flush=True)
    arms = {"k_flat": None, "xcd_weighted": m}

    def set_arm(name):
        wts = arms[name]
        engine.tune_xcd_weights(wts, a.period if wts else 0)

    for name in arms:
        set_arm(name)
        run()
        res, per = traced(run, n)
        kern = last_kernel()
        set_arm("k_flat")
        ends = [p["end_us"] for p in per.values()]
        print(json.dumps({"step": "trace", "arm": name, "kernel": kern, "results_equal": bool(torch.equal(res, ref)),
                          "xcd_end_spread_us": round(max(ends) - min(ends), 2), "span_us": round(max(ends), 2),
                          "per_xcd": per}), flush=True)
    med = {k: [] for k in arms}
    for r in range(a.rounds):
        for name in (arms if r % 2 == 0 else reversed(list(arms))):
            set_arm(name)
            run()
            med[name].append(timed(run, a.iters))
            assert torch.equal(out, ref), name
            set_arm("k_flat")
    summ = {k: round(statistics.median(v), 4) for k, v in med.items()}
    print(json.dumps({"step": "ab", "packets": n, "rounds": a.rounds, "iters": a.iters, "median_ms": summ,
                      "per_round_ms": {k: [round(x, 4) for x in v] for k, v in med.items()},
                      "weighted_vs_default": round(summ["xcd_weighted"] / summ["k_flat"] - 1, 4),
                      "frac_of_8TBs": {k: round(n * (w.length + 2) / (v / 1e3) / 8e12, 4) for k, v in summ.items()}}),
          flush=True)


if __name__ == "__main__":
    main()

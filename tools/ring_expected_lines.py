#!/usr/bin/env python3
"""The HBM bytes each RX ring of tools/rx_device_bench.py must move, from its
frame-length mix alone: a line model to set beside the
PMC-measured traffic of tools/pmc_rx.sh.

    python tools/ring_expected_lines.py [--packets 8388608]  > profiles/r06_ring_expected_lines.jsonl

Model.  A frame sits at the start of its slot (slot strides are multiples of
128 B, so every frame starts on a 128-B line) and L2 fetches whole 128-B lines
from HBM: a frame of F bytes costs ceil(F / 128) lines, 128 B each, whatever
part of the last line it uses.  Beside the frames the verifier reads the u16
slot lengths (2 B per slot, one contiguous stream) and writes one verdict byte
per slot (whole lines of a block's 64 verdicts).  Nothing else: the header
windows are captured from the frame stream, and no byte of a slot past its
frame is requested.  Algorithmic bytes (rx_device_bench's fraction): frame
bytes + 1 verdict byte per slot.

Frame mix (engine.gen_rx_frames / gen_rx_ring): L4 lengths fixed per ring, or
cfg4's Zipf lengths (64-9,000 B, the generator twin in oracle/pipck_oracle.c)
for the sparse ring; each frame is TCP/IPv4 or UDP/IPv4 (20-B header) with
probability 3/4 and TCP/IPv6 (40 B) with 1/4 -- the expectation over that
draw is what is computed.  Frame sizes follow pip's own segments: a pure ACK
or a short segment is a 40-60-B TCP/IPv4 frame
(pip/protocol/pip_tcp_private.cpp:12-22 builds 20-B TCP headers plus options),
so the short rings' ~120-240-B frames are the regime where the last partial
line dominates.
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

LINE = 128
RINGS = (("ring_sparse_9216", 9216, 0, 1), ("ring_dense_1536", 1536, 1480, 1), ("ring_dense_9216", 9216, 8900, 2),
         ("ring_short_2048", 2048, 200, 1), ("ring_short_1024", 1024, 100, 1))
HDR = ((20, 0.75), (40, 0.25))  # (IP header bytes, probability): kinds 0-2 IPv4, kind 3 IPv6


def expected(l4: np.ndarray) -> dict:
    n = l4.size
    frame_bytes = sum(p * float((l4 + h).sum()) for h, p in HDR)
    lines = sum(p * float(((l4 + h + LINE - 1) // LINE).sum()) for h, p in HDR)
    hbm = lines * LINE + 2 * n + n  # frame lines + u16 lengths + verdict bytes
    algo = frame_bytes + n
    return {"frames": n, "frame_bytes": round(frame_bytes), "lines_per_frame": round(lines / n, 4),
            "expected_hbm_bytes": round(hbm), "algorithmic_bytes": round(algo),
            "expected_ratio": round(hbm / algo, 4)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=8 << 20)
    a = ap.parse_args()
    zipf = None
    for tag, stride, l4_len, div in RINGS:
        n = a.packets // div
        if l4_len:
            l4 = np.full(n, l4_len, dtype=np.int64)
        else:
            if zipf is None or zipf.size < n:
                from oracle.oracle import Oracle

                orc = Oracle()
                seed = 0
                from pip_amd.workloads import BY_CFG

                seed = BY_CFG[4].seed
                zipf = orc.zipf_lengths(seed, 0, n).astype(np.int64)
            l4 = zipf[:n]
        print(json.dumps({"what": tag, "stride": stride, "l4_len": l4_len or "zipf 64-9000 (cfg4)", **expected(l4)}),
              flush=True)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Summarise tools/hdr_spread.sh runs: per box (gpurun_out/hdr_spread_<TAG>) and arm,
the median kernel time, HBM bytes per launch from FETCH_SIZE (x2, the gfx950
correction) and WRITE_SIZE (KiB), and the SQ counters of the k_hdr dispatch.
    python tools/hdr_spread_summary.py s1 s2 [...] > profiles/r04_hdr_result_stream.jsonl"""
import collections
import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def counters(d: Path) -> dict:
    by = collections.defaultdict(dict)
    for r in csv.DictReader(open(d / "run_counter_collection.csv")):
        if "k_hdr" in r["Kernel_Name"]:
            by[int(r["Dispatch_Id"])][r["Counter_Name"]] = by[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0.0) + \
                float(r["Counter_Value"])
    return by[max(by)] if by else {}


for tag in sys.argv[1:]:
    base = ROOT / "gpurun_out" / f"hdr_spread_{tag}"
    ab = json.loads((base / "ab.jsonl").read_text().strip().splitlines()[-1])
    n = ab["headers"]
    for arm, ms in ab["median_ms"].items():
        f = counters(base / f"{arm}_FETCH_SIZE").get("FETCH_SIZE", 0.0)
        w = counters(base / f"{arm}_WRITE_SIZE").get("WRITE_SIZE", 0.0)
        sq = counters(base / f"{arm}_SQ_WAVES")
        rd, wr = 2 * f * 1024, w * 1024
        print(json.dumps({"box": tag, "arm": arm, "headers": n, "median_ms": ms,
                          "frac_of_8TBs_algorithmic": round(n * 22 / (ms / 1e3) / 8e12, 4),
                          "hbm_read_bytes": round(rd), "hbm_write_bytes": round(wr),
                          "read_per_header": round(rd / n, 3), "write_per_header": round(wr / n, 3),
                          "hbm_TBps": round((rd + wr) / (ms / 1e3) / 1e12, 3),
                          "sq": {k: int(v) for k, v in sorted(sq.items())},
                          "wait_frac": round(sq.get("SQ_WAIT_INST_ANY", 0) / max(sq.get("SQ_WAVE_CYCLES", 1), 1), 4)}))

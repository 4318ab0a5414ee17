#!/usr/bin/env python3
"""Condense tools/pmc_rx.sh runs into profiles/traffic_rx_<workload>.json and
profiles/<tag>_rx_pmc_summary.md.

    python tools/pmc_rx_summary.py r05

Per workload: the RX kernel's dispatches (k_packedb_rx for the byte-packed
frames, k_ring for the rings), HBM bytes per launch = 2 x FETCH_SIZE x 1024 +
WRITE_SIZE x 1024 (gfx950: FETCH_SIZE counts half the bytes of 16-B-per-lane
streams, MI355X_MICROARCH.md HBM section; WRITE_SIZE exact for those), against
the algorithmic bytes tools/rx_device_bench.py uses for its fraction (frame
bytes read + the 1-B verdict per frame written).  The rocprof kernel-trace
duration of the same kernel is recorded beside it.
"""
from __future__ import annotations

import csv
import hashlib
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def rows(p: Path):
    with open(p) as f:
        return list(csv.DictReader(f))


def find(d: Path, suffix: str) -> Path | None:
    hits = sorted(d.rglob(f"*{suffix}"))
    return hits[0] if hits else None


def main() -> None:
    tag = sys.argv[1] if len(sys.argv) > 1 else "r05"
    lib = ROOT / "pip_amd" / "lib" / "libpipck.so"
    sha = hashlib.sha256(lib.read_bytes()).hexdigest() if lib.exists() else None
    md = [f"# {tag}: RX verifier PMC passes (tools/pmc_rx.sh)", "",
          "HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KB x 1024), per dispatch of the RX kernel; "
          "algorithmic = frame bytes read + 1 verdict byte per frame (tools/rx_device_bench.py).", "",
          "Expected = the line model of tools/ring_expected_lines.py (profiles/r06_ring_expected_lines.jsonl): "
          "every 128-B line a frame touches, fetched whole, + 2 B of slot length + the 1-B verdict per slot "
          "(rings only; the byte-packed frames share lines with their neighbours).", "",
          "| workload | kernel | frames | algorithmic B | HBM B (PMC) | ratio | expected lines/frame | expected ratio "
          "| measured / expected | rocprof median ms | frac of 8 TB/s |",
          "|---|---|---|---|---|---|---|---|---|---|---|"]
    exp = {}
    ef = ROOT / "profiles" / "r06_ring_expected_lines.jsonl"
    if ef.exists():
        exp = {d["what"]: d for d in map(json.loads, ef.read_text().splitlines())}
    for d in sorted((ROOT / "gpurun_out").glob(f"pmc_rx_{tag}_*")):
        wl = d.name[len(f"pmc_rx_{tag}_"):]
        lines = [json.loads(x) for x in (d / "trace.jsonl").read_text().splitlines() if x.startswith("{")]
        line = [x for x in lines if x["what"] == ("rx_verify_device" if wl == "packed" else wl)][-1]
        kname = line["last_kernel"].split("(")[0]
        algo = line["frame_bytes"] + line["packets"]

        def counter(sub: str, name: str) -> float:
            p = find(d / sub, "counter_collection.csv")
            vals = [float(r["Counter_Value"]) for r in rows(p)
                    if r["Kernel_Name"].split("(")[0] == kname and r["Counter_Name"] == name] if p else []
            return statistics.mean(vals) if vals else float("nan")

        fetch, write = counter("pmc_fetch", "FETCH_SIZE"), counter("pmc_write", "WRITE_SIZE")
        tr = find(d / "trace", "kernel_trace.csv")
        durs = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows(tr)
                      if r["Kernel_Name"].split("(")[0] == kname) if tr else []
        med = statistics.median(durs) if durs else float("nan")
        hbm = 2 * fetch * 1024 + write * 1024
        t = {"workload": wl, "tag": tag, "kernel": kname, "lib_sha256": sha, "frames": line["packets"],
             "frame_bytes": line["frame_bytes"], "algorithmic_bytes_per_launch": algo,
             "fetch_size_kb": fetch, "write_size_kb": write, "hbm_bytes_per_launch": int(hbm),
             "traffic_over_algorithmic": round(hbm / algo, 4), "rocprof_dispatches": len(durs),
             "rocprof_median_ns": med, "frac_by_rocprof": round(algo / (med / 1e9) / 8e12, 4),
             "correction": "hbm = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE counts 1/2 of wide streams)"}
        e = exp.get(wl)
        if e and e["frames"] == line["packets"]:
            t["expected_lines_per_frame"] = e["lines_per_frame"]
            t["expected_ratio"] = e["expected_ratio"]
            ecols = f"{e['lines_per_frame']:.3f} | {e['expected_ratio']:.4f} | {hbm / algo / e['expected_ratio']:.4f}"
        else:
            ecols = "- | - | -"
        md.append(f"| {wl} | `{kname}` | {line['packets']:,} | {algo:,} | {int(hbm):,} | {hbm / algo:.4f} | "
                  f"{ecols} | {med / 1e6:.4f} | {t['frac_by_rocprof']:.3f} |")
        (ROOT / "profiles" / f"traffic_rx_{wl if wl != 'packed' else 'rx_verify_device'}.json").write_text(
            json.dumps(t, indent=1) + "\n")
    md += ["", f"libpipck.so sha256 `{sha}`", ""]
    (ROOT / "profiles" / f"{tag}_rx_pmc_summary.md").write_text("\n".join(md))
    print("\n".join(md))


if __name__ == "__main__":
    main()

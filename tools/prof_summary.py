#!/usr/bin/env python3
"""Condense a tools/profile.sh run into committed files under profiles/.

    python tools/prof_summary.py gpurun_out/prof_r01_cfg5 r01 cfg5

Writes profiles/<tag>_<wl>_kernel_stats.csv (rocprofv3 --stats, verbatim),
profiles/<tag>_<wl>_pmc.csv (counter rows of the dominant kernel),
profiles/<tag>_<wl>_summary.md and profiles/traffic_<wl>.json, which bench.py
reads for roofline.traffic.

HBM bytes per launch = 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024: on gfx950
FETCH_SIZE (KB) counts half the bytes of a wide (16 B/lane) coalesced stream
(MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact for 16-B stores and
is negligible here (2 B of results per packet).
"""
from __future__ import annotations

import csv
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def rows(path: Path):
    with open(path) as f:
        return list(csv.DictReader(f))


def find(d: Path, suffix: str) -> Path:
    hits = sorted(d.rglob(f"*{suffix}"))
    if not hits:
        raise FileNotFoundError(f"no *{suffix} under {d}")
    return hits[0]


def main() -> None:
    out_dir, tag, wl = Path(sys.argv[1]), sys.argv[2], sys.argv[3]
    prof = ROOT / "profiles"
    prof.mkdir(exist_ok=True)
    stats_p = find(out_dir / "trace", "kernel_stats.csv")
    stats = rows(stats_p)
    # the measured kernel: the costliest one that is not the batch generator (which can
    # outweigh the timed launches when a large cfg1 batch is generated once)
    top = max([r for r in stats if "k_gen" not in r["Name"]] or stats, key=lambda r: float(r["TotalDurationNs"]))
    kname = top["Name"]
    (prof / f"{tag}_{wl}_kernel_stats.csv").write_text(stats_p.read_text())

    bench = json.loads((out_dir / "trace.json").read_text().strip().splitlines()[-1])
    algo = bench["roofline"]["algorithmic_bytes_per_launch"]

    def counter(name: str, sub: str) -> tuple[float, list[dict]]:
        p = find(out_dir / sub, "counter_collection.csv")
        rs = [r for r in rows(p) if r.get("Kernel_Name") == kname and r.get("Counter_Name") == name]
        vals = [float(r["Counter_Value"]) for r in rs]
        return (statistics.mean(vals) if vals else float("nan")), rs

    fetch_kb, frows = counter("FETCH_SIZE", "pmc_fetch")
    write_kb, wrows = counter("WRITE_SIZE", "pmc_write")
    with open(prof / f"{tag}_{wl}_pmc.csv", "w", newline="") as f:
        keep = ["Kernel_Name", "Counter_Name", "Counter_Value", "Grid_Size", "Workgroup_Size", "VGPR_Count",
                "SGPR_Count", "LDS_Block_Size"]
        w = csv.DictWriter(f, fieldnames=keep, extrasaction="ignore")
        w.writeheader()
        for r in frows + wrows:
            w.writerow(r)
    hbm = 2 * fetch_kb * 1024 + write_kb * 1024
    # per-dispatch durations of the bench's TIMED launches (the last `steps` dispatches of
    # the kernel in the trace): --stats' AverageNs also counts the warm-up launches, which
    # run back to back on a cold chip and are a few % slower
    all_ns = float(top["AverageNs"])
    avg_ns = all_ns
    try:
        tr = [r for r in rows(find(out_dir / "trace", "kernel_trace.csv")) if r["Kernel_Name"] == kname]
        tr.sort(key=lambda r: int(r["Start_Timestamp"]))
        timed = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr[-int(bench["steps"]):]]
        if timed:
            avg_ns = statistics.mean(timed)
            med_ns = statistics.median(timed)
    except FileNotFoundError:
        timed = []
    if not timed:
        med_ns = avg_ns
    bench_kernel = bench["roofline"].get("kernel")
    if bench_kernel != kname:
        print(f"WARNING: rocprof's dominant kernel {kname!r} is not the one the bench line timed "
              f"({bench_kernel!r}); bench.py will not attach this traffic", file=sys.stderr)
    traffic = {"workload": wl, "tag": tag, "kernel": kname, "lib_sha256": bench["roofline"].get("lib_sha256"),
               "bench_kernel_matches": bench_kernel == kname,
               "fetch_size_kb": fetch_kb, "write_size_kb": write_kb,
               "hbm_bytes_per_launch": int(hbm), "algorithmic_bytes_per_launch": algo,
               "arena_stride": bench["config"]["arena_stride"], "packets": bench["config"]["packets_per_gpu"],
               "traffic_over_algorithmic": round(hbm / algo, 4), "rocprof_avg_ns": avg_ns,
               "bench_event_kernel_ms": bench["roofline"]["kernel_ms"],
               "rocprof_vs_bench_event": round(avg_ns / 1e6 / bench["roofline"]["kernel_ms"], 4),
               "rocprof_avg_ns_all_calls": all_ns, "rocprof_timed_dispatches": len(timed),
               "rocprof_timed_median_ns": med_ns if timed else None,
               "correction": "hbm = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE counts 1/2 of wide streams)"}
    # a tag with a size suffix (TAG=r02_268435456) profiles a non-default batch size:
    # keep it beside, not over, the default-size traffic file bench.py reads
    sfx = f"_{tag.split('_', 1)[1]}" if "_" in tag else ""
    (prof / f"traffic_{wl}{sfx}.json").write_text(json.dumps(traffic, indent=1) + "\n")
    md = [f"# {tag} {wl}: rocprofv3 summary", "",
          f"Command: `tools/profile.sh` (TAG={tag} WL={wl}) on one MI355X; bench line of the trace pass:", "",
          "```", json.dumps(bench), "```", "",
          "| kernel | calls | avg us (rocprof) | share |", "|---|---|---|---|"]
    for r in sorted(stats, key=lambda r: -float(r["TotalDurationNs"]))[:6]:
        md.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                  f"{float(r['Percentage']):.2f}% |")
    md += ["", f"Dominant kernel: `{kname}`", "",
           f"* libpipck.so sha256 `{bench['roofline'].get('lib_sha256')}` (bench.py attaches this traffic "
           f"only to lines of this kernel and build)",
           f"* rocprof kernel trace, the {len(timed)} timed dispatches: mean {avg_ns / 1e6:.4f} ms, median "
           f"{(med_ns if timed else avg_ns) / 1e6:.4f} ms; --stats average over all {top['Calls']} calls (warm-up "
           f"included) {all_ns / 1e6:.4f} ms",
           f"* bench per-dispatch HIP-event median {bench['roofline']['kernel_ms']} ms (back-to-back mean "
           f"{bench['roofline'].get('kernel_ms_b2b_mean')} ms)",
           f"* algorithmic bytes per launch {algo:,} (L + 2 per packet)",
           f"* FETCH_SIZE {fetch_kb:,.0f} KB, WRITE_SIZE {write_kb:,.0f} KB per launch",
           f"* HBM bytes per launch (2 x FETCH + WRITE) {hbm:,.0f} = {hbm / algo:.3f} x algorithmic",
           f"* achieved (median timed dispatch) {algo / (med_ns / 1e9) / 1e9:,.1f} GB/s algorithmic = "
           f"{algo / (med_ns / 1e9) / 8e12:.3f} of 8 TB/s; (mean) {algo / (avg_ns / 1e9) / 1e9:,.1f} GB/s = "
           f"{algo / (avg_ns / 1e9) / 8e12:.3f}", ""]
    (prof / f"{tag}_{wl}_summary.md").write_text("\n".join(md))
    print("\n".join(md))


if __name__ == "__main__":
    main()

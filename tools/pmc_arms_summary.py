#!/usr/bin/env python3
"""Summarise tools/pmc_arms.sh: mean FETCH_SIZE / WRITE_SIZE (KB) per dispatch of the
dominant pipck kernel per arm -> HBM bytes per launch (2 x FETCH + WRITE, gfx950)."""
import csv
import json
import statistics
import sys
from pathlib import Path

d = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_arms")
for arm in (d / "arm_names.txt").read_text().split():
    res = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = []
        for f in (d / f"{arm}_{c}").rglob("*counter_collection.csv"):
            rows += [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == c and "pipck::k_" in r["Kernel_Name"]
                     and "k_gen" not in r["Kernel_Name"]]
        top = max({r["Kernel_Name"] for r in rows}, key=lambda k: sum(float(r["Counter_Value"]) for r in rows
                                                                     if r["Kernel_Name"] == k))
        res[c] = statistics.mean(float(r["Counter_Value"]) for r in rows if r["Kernel_Name"] == top)
        res["kernel"] = top.split("(")[0]
    line = json.loads((d / f"{arm}_FETCH_SIZE.jsonl").read_text().splitlines()[-1])
    algo = line.get("bytes") or line["gbytes"] * 1e9
    hbm = 2 * res["FETCH_SIZE"] * 1024 + res["WRITE_SIZE"] * 1024
    print(json.dumps({"arm": arm, "kernel": res["kernel"], "workload": line["workload"], "packets": line["packets"],
                      "fetch_kb": res["FETCH_SIZE"], "write_kb": res["WRITE_SIZE"], "hbm_bytes": int(hbm),
                      "algorithmic_bytes_approx": int(algo), "traffic_over_algorithmic": round(hbm / algo, 4)}))

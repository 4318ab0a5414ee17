#!/usr/bin/env python3
"""Per-kernel instruction mix and stall split from a tools/sq_profile.sh run
(run here, on the merged CSVs).

    python tools/sq_summary.py gpurun_out/sq_cfg4 [kernel-substring]

Per 1 KiB row (one 64-lane x 16 B VMEM read instruction): VALU / SALU / LDS
instructions; per wave cycle: parked on s_waitcnt (WAIT_ANY), issue-stalled
(WAIT_INST_ANY), issuing (ACTIVE_INST_ANY), VALU and LDS busy.
"""
import collections
import csv
import sys
from pathlib import Path


def load(path, pat):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    if not Path(path).exists():
        return agg
    with open(path) as f:
        for r in csv.DictReader(f):
            if pat in r["Kernel_Name"]:
                agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
    return agg


def main():
    d = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "pipck::k_"
    a = load(f"{d}/pmc/run_counter_collection.csv", pat)
    b = load(f"{d}/pmc2/run_counter_collection.csv", pat)
    for k, v in a.items():
        rows = v.get("SQ_INSTS_VMEM_RD", 0.0)
        if not rows:
            continue
        line = (f"{k}: VALU/row {v['SQ_INSTS_VALU'] / rows:.1f}  SALU/row {v['SQ_INSTS_SALU'] / rows:.1f}  "
                f"LDS/row {v['SQ_INSTS_LDS'] / rows:.2f}  rows {rows:.3g}")
        w = b.get(k)
        cyc = v.get("SQ_WAVE_CYCLES", 0.0)
        if w and cyc:
            # pass 2 ran the same launches: scale by its own VMEM count in case the launch count differs
            sc = rows / max(w.get("SQ_INSTS_VMEM_RD", rows), 1.0)
            line += ("  | of wave cycles: waitcnt {:.2f}  issue-stall {:.2f}  active {:.2f}  VALU {:.2f}  "
                     "LDS {:.2f}  LDS-issue-stall {:.2f}").format(
                w["SQ_WAIT_ANY"] * sc / cyc, v["SQ_WAIT_INST_ANY"] / cyc, w["SQ_ACTIVE_INST_ANY"] * sc / cyc,
                w["SQ_ACTIVE_INST_VALU"] * sc / cyc, w["SQ_ACTIVE_INST_LDS"] * sc / cyc,
                w["SQ_WAIT_INST_LDS"] * sc / cyc)
        print(line)


if __name__ == "__main__":
    main()

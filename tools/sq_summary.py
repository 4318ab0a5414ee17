#!/usr/bin/env python3
"""Per-kernel instruction mix from a tools/sq_profile.sh run (run here, on the merged CSV).

    python tools/sq_summary.py gpurun_out/sq_cfg4 [kernel-substring]

Per 1 KiB row (one 64-lane x 16 B VMEM read instruction): VALU / SALU / LDS
instructions, plus the fraction of wave cycles spent waiting.
"""
import collections
import csv
import sys


def main():
    d = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "pipck::k_"
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    with open(f"{d}/pmc/run_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            if pat in r["Kernel_Name"]:
                agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in agg.items():
        rows = v.get("SQ_INSTS_VMEM_RD", 0.0)
        if not rows:
            continue
        print(f"{k}: VALU/row {v['SQ_INSTS_VALU'] / rows:.1f}  SALU/row {v['SQ_INSTS_SALU'] / rows:.1f}  "
              f"LDS/row {v['SQ_INSTS_LDS'] / rows:.2f}  wait/wave-cycles "
              f"{v['SQ_WAIT_INST_ANY'] / max(v['SQ_WAVE_CYCLES'], 1):.2f}  rows {rows:.3g}")


if __name__ == "__main__":
    main()

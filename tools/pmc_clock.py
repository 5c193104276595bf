#!/usr/bin/env python3
"""Summarise tools/pmc_clock.sh: per variant and fused kernel, the average wall time per
dispatch (kernel trace), effective clock GRBM_GUI_ACTIVE / 8 / wall, and SQ activity ratios."""
import csv
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_summary import bench_name  # noqa: E402


def find(d, suffix):
    return next(Path(d).rglob(f"*{suffix}"))


def main(out, variants):
    for v in variants:
        name = v.split(":")[0]
        d = Path(out) / name
        dur = {}
        for r in csv.DictReader(open(find(d, "kernel_trace.csv"))):
            dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        acc = defaultdict(lambda: defaultdict(float))
        seen = defaultdict(set)
        for r in csv.DictReader(open(find(d, "counter_collection.csv"))):
            k = bench_name(r["Kernel_Name"])
            if k not in ("fused_reverse", "fused_apply"):
                continue
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            if r["Dispatch_Id"] not in seen[k]:
                seen[k].add(r["Dispatch_Id"])
                acc[k]["wall"] += dur.get(r["Dispatch_Id"], 0.0)
        for k, c in sorted(acc.items()):
            n = len(seen[k])
            wall = c["wall"]
            clk = c["GRBM_GUI_ACTIVE"] / 8 / wall / 1e9 if wall else 0
            print(f"{name:8s} {k:14s} n={n:3d} wall {wall / n * 1e3:7.3f} ms  clock {clk:5.2f} GHz  "
                  f"VALU-active/busy {c['SQ_ACTIVE_INST_VALU'] / max(c['SQ_BUSY_CYCLES'], 1):6.2f}  "
                  f"VALU insts/wave-cycle {c['SQ_INSTS_VALU'] / max(c['SQ_WAVE_CYCLES'], 1):.4f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])

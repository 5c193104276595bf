#!/usr/bin/env python3
"""rocprofv3 kernel stats aggregated by the bench's kernel names (specialized pass kernels are
one symbol per program): calls, total and average duration per bench name.
usage: python tools/r5/stats_by_name.py <trace_kernel_stats.csv> <out.csv>"""
import csv
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from pmc_summary import bench_name  # noqa: E402

calls, total = defaultdict(int), defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    k = bench_name(r["Name"]) or r["Name"][:40]
    calls[k] += int(r["Calls"])
    total[k] += float(r["TotalDurationNs"])
allt = sum(total.values())
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["bench_name", "calls", "total_ms", "avg_ms", "share"])
    for k in sorted(total, key=lambda k: -total[k]):
        w.writerow([k, calls[k], round(total[k] / 1e6, 4), round(total[k] / calls[k] / 1e6, 5),
                    round(total[k] / allt, 4)])
print(open(sys.argv[2]).read())

#!/usr/bin/env python3
"""Aggregate a rocprofv3 --stats kernel table by the bench's kernel names (tools/pmc_summary.py
bench_name): the specialized passes (qdc_spec_<hash> reverse, qdc_specf_<hash> forward: one
symbol per pass program) count with their interpreted kernels as fused_reverse / fused_apply.  usage: trace_agg.py <trace_kernel_stats.csv>"""
import csv
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_summary import bench_name  # noqa: E402

calls, ns = defaultdict(int), defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    k = bench_name(r["Name"]) or r["Name"][:60]
    calls[k] += int(r["Calls"])
    ns[k] += float(r["TotalDurationNs"])
tot = sum(ns.values())
print("kernel,calls,total_ms,avg_ms,share")
for k in sorted(ns, key=lambda x: -ns[x]):
    print(f"{k},{calls[k]},{ns[k] / 1e6:.3f},{ns[k] / calls[k] / 1e6:.4f},{ns[k] / tot:.4f}")

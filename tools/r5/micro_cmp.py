"""Compare single-gate sweep logs (bench.py --micro): one column per log, % of 8 TB/s."""
import re
import sys


def parse(f):
    d = {}
    for line in open(f):
        m = re.match(r"(q[12] [\d,]+)\s+(\S+)\s+n=\s*\d+\s+([\d.]+) ms\s+([\d.]+) GB/s\s+([\d.]+)%", line)
        if m:
            d[(m.group(1), m.group(2))] = float(m.group(5))
    return d


files = sys.argv[1:]
ds = [parse(f) for f in files]
only = None
print(" " * 30 + " ".join(f"{f.split('micro_')[-1][:8]:>8s}" for f in files))
for k in ds[0]:
    if k[1] in ("copy", "density_q1", "inject_diag", "apply_q2_diag"):
        continue
    print(f"{k[0]:10s} {k[1]:18s}" + " ".join(f"{d.get(k, 0):8.1f}" for d in ds))
for i, d in enumerate(ds):
    gate = {k: v for k, v in d.items() if k[1].startswith(("apply_", "reverse_"))}
    w = min(gate, key=gate.get)
    print(files[i], "min", w, gate[w], "cells<75:", sum(v < 75 for v in gate.values()))

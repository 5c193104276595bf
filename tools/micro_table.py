"""Summarise `bench.py --micro` output: % of the 8 TB/s spec per kernel and gate position."""
import re
import sys
from collections import OrderedDict

rows = OrderedDict()
cols = []
for line in open(sys.argv[1]):
    m = re.match(r"(q\d \S+)\s+(\S+)\s+n=\s*\d+\s+([\d.]+) ms\s+([\d.]+) GB/s", line)
    if not m:
        continue
    label, k, ms, gbs = m.group(1), m.group(2), float(m.group(3)), float(m.group(4))
    if k in ("copy", "finalize"):
        continue
    rows.setdefault(label, {})[k] = gbs / 8000 * 100
    if k not in cols:
        cols.append(k)
print("%-10s" % "gate" + "".join("%16s" % c for c in cols))
for label, d in rows.items():
    print("%-10s" % label + "".join(("%15.1f%%" % d[c]) if c in d else "%16s" % "-" for c in cols))

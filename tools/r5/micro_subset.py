"""Single-gate sweep (bench.py micro) over a subset of placements: q1 positions and q2 pairs
from the command line, e.g.  python tools/r5/micro_subset.py --q1 12,20,24 --q2 5:20,26:27"""
import argparse
import sys

sys.path.insert(0, ".")
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--q1", default="")
ap.add_argument("--q2", default="")
ap.add_argument("--qubits", type=int, default=28)
a = ap.parse_args()
args = bench.parse([])
args.qubits = a.qubits
q1 = [int(x) for x in a.q1.split(",") if x]
q2 = [tuple(int(y) for y in x.split(":")) for x in a.q2.split(",") if x]
bench.micro(args, a.qubits, verbose=True, q1_positions=q1, q2_pairs=q2)

#!/usr/bin/env python3
"""Per-kernel sums of the SQ counters collected by tools/pmc_sq.sh (averaged per launch)."""
import csv
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from pmc_summary import bench_name  # noqa: E402


def main(root):
    root = Path(root)
    for run in sorted({p.name.split("_p")[0] for p in root.glob("rq*_p*") if p.is_dir()}):
        tot = defaultdict(lambda: defaultdict(float))
        cnt = defaultdict(lambda: defaultdict(int))
        for d in sorted(root.glob(run + "_p*")):
            for f in d.rglob("*counter_collection.csv"):
                for r in csv.DictReader(open(f)):
                    k = bench_name(r["Kernel_Name"]) or r["Kernel_Name"][:30]
                    tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
                    cnt[k][r["Counter_Name"]] += 1
        print("==", run)
        for k in sorted(tot):
            if not k.startswith("fused"):
                continue
            c = {n: tot[k][n] / max(cnt[k][n], 1) for n in tot[k]}
            print(k, " ".join(f"{n}={v:.4g}" for n, v in sorted(c.items())))


if __name__ == "__main__":
    main(sys.argv[1])

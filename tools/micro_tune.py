"""Single-gate kernel knobs at the weak cells of the bench sweep (bench.py micro): each
configuration (QDC_* environment, read when a circuit is created) over the selected cases,
repeated in alternating order; prints one table row per (config, case, kernel) with the median
fraction of the 8 TB/s HBM peak over the repetitions."""
import argparse
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=28)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--q1", default="1,3,20,22,24")
    ap.add_argument("--q2", default="5:20,26:27,14:13")
    ap.add_argument("--cfgs", required=True, help="space-separated; '-' = defaults; k=v,k=v")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    args = bench.parse([])
    args.qubits = a.qubits
    q1 = [int(x) for x in a.q1.split(",") if x]
    q2 = [tuple(int(y) for y in x.split(":")) for x in a.q2.split(",") if x]
    cfgs = a.cfgs.split()
    res = {}
    for rep in range(a.reps):
        order = cfgs if rep % 2 == 0 else cfgs[::-1]
        for cfg in order:
            kv = {} if cfg == "-" else dict(x.split("=", 1) for x in cfg.split(","))
            old = {k: os.environ.get(k) for k in kv}
            os.environ.update(kv)
            try:
                rows = bench.micro(args, a.qubits, verbose=False, q1_positions=q1, q2_pairs=q2)
            finally:
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
            for label, kern, _, ms, gbs in rows:
                res.setdefault((cfg, label, kern), []).append(gbs / bench.HBM_PEAK_GBS)
            print(f"[tune] rep {rep} {cfg} done", flush=True)
    table = []
    for (cfg, label, kern), v in sorted(res.items(), key=lambda kv: (kv[0][1], kv[0][2], kv[0][0])):
        med = sorted(v)[len(v) // 2]
        table.append({"cfg": cfg, "case": label, "kernel": kern, "frac": round(med, 4),
                      "all": [round(x, 4) for x in v]})
        print(f"{label:10s} {kern:16s} {cfg:40s} {med:6.1%}  {' '.join(f'{x:.3f}' for x in v)}")
    if a.out:
        Path(a.out).write_text(json.dumps(table, indent=1))


if __name__ == "__main__":
    main()

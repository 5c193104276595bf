#!/usr/bin/env python3
"""Per-pass time model of the fused reverse sweep.

Joins a rocprofv3 kernel trace (per-dispatch start / end) of the C2 bench step with the
sources of the specialized kernels the same program launches (a dry run of the bench's C2
program: QDC_PRECOMPILE_DUMP=<dir> q.precompile(...), see main()), counts per reverse pass its
Gamma stages, stages and relayouts from the kernel source, fits

    t_pass ~= max(skeleton, a * gamma_stages + b * relayouts + c)

by least squares over the compute-bound passes, and compares the sum over a step with the
balanced bound (the same work spread so that no pass idles below the memory skeleton).

usage: pass_model.py TRACE_CSV [DUMP_DIR]
"""
import csv
import re
import sys
from collections import defaultdict
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]


def dump_sources(out):
    """The bench's C2 program (n = 28, 20 layers, seed 24, world 1): dry-run forward + backward,
    every specialized kernel's source to out/<name>.hip."""
    import os
    sys.path[:0] = [str(ROOT), str(ROOT / "differentiable-quantum-circuit-cuda_amd")]
    os.environ["QDC_PRECOMPILE_DUMP"] = str(out)
    os.environ["QDC_PRECOMPILE_COUNT"] = "1"
    import quantum_differentiable_circuit as q
    from quantum_differentiable_circuit import workloads as W
    ins, var = W.layered_circuit(28, 20, 24)
    instr = [(k, *p) for k, p in ins]
    vg = [np.ascontiguousarray(g, dtype=np.complex64) for g in var]
    cots = [np.diag([1.0, -1.0]).astype(np.complex64) for k, _ in ins if k == W.DIFF_Q1_DENSITY]
    out.mkdir(parents=True, exist_ok=True)
    return q.precompile(28, instr, [], vg, cots, world=1, precision="f32")


def features(src):
    two = "(xf, xb, E" in src or "qdc::cx (&xf)" in src
    stages = len(re.findall(r"rq_(?:q1|q2|diag)<", src))
    gamma = len(re.findall(r", true, &E\.accw", src))
    relay = src.count("{ constexpr uint32_t")
    q2 = len(re.findall(r"rq_q2<", src))
    return {"two": two, "stages": stages, "gamma": gamma, "relayouts": relay, "q2": q2}


def main():
    trace = Path(sys.argv[1])
    dump = Path(sys.argv[2]) if len(sys.argv) > 2 else Path("/tmp/qdc_pass_model_src")
    if not (dump / "order.txt").exists():
        print(f"dry run: {dump_sources(dump)} kernels -> {dump}", file=sys.stderr)
    feat = {}
    for f in dump.glob("*.hip"):
        feat[f.stem] = features(f.read_text())
    rows = []
    with open(trace) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # kernel names under rocprofv3 can differ from the dry run's (the fingerprint sees the
    # profiler's environment): map them by first use, the dry run's order.txt order
    order = (dump / "order.txt").read_text().split()
    first = []
    for _, _, name in rows:
        base = name.split("(")[0].strip()
        if base.startswith("qdc_spec") and base not in first:
            first.append(base)
    if set(first) <= set(feat):
        alias = {k: k for k in first}
    else:
        assert len(first) == len(order), (len(first), len(order))
        for a, b in zip(first, order):
            assert a.split("_")[1] == b.split("_")[1], (a, b)  # spec / specf kinds in step
        alias = dict(zip(first, order))
    per = defaultdict(list)
    for s, e, name in rows:
        base = alias.get(name.split("(")[0].strip())
        if base in feat:
            per[base].append((e - s) * 1e-6)
    # the timed steps' dispatches: the median duration of each reverse kernel (launched once per
    # step; the first launches are the warm-up)
    rev = [(k, float(np.median(v))) for k, v in per.items() if feat[k]["two"]]
    fwd = [(k, float(np.median(v))) for k, v in per.items() if not feat[k]["two"]]
    print(f"reverse kernels in trace: {len(rev)}, forward: {len(fwd)}")
    t = np.array([x[1] for x in rev])
    G = np.array([feat[k]["gamma"] for k, _ in rev], float)
    R = np.array([feat[k]["relayouts"] for k, _ in rev], float)
    S = np.array([feat[k]["stages"] for k, _ in rev], float)
    print(f"per-pass ms: min {t.min():.3f} median {np.median(t):.3f} max {t.max():.3f}, sum {t.sum():.2f}")
    skel = float(sys.argv[3]) if len(sys.argv) > 3 else 1.72  # r5 ablation: memory skeleton
    cb = t > skel * 1.1
    X = np.stack([G, R, np.ones_like(G)], 1)
    coef, *_ = np.linalg.lstsq(X[cb], t[cb], rcond=None)
    pred = np.maximum(skel, X @ coef)
    resid = t - pred
    print(f"fit over {cb.sum()} compute-bound passes: t = {coef[0]:.4f} ms/Gamma-stage + "
          f"{coef[1]:.4f} ms/relayout + {coef[2]:.4f} ms; rms residual {np.sqrt((resid ** 2).mean()):.3f} ms")
    comp = X @ coef
    slack = np.maximum(0, skel - comp).sum()  # compute capacity idle below the skeleton
    total = t.sum()
    bound = max(skel * len(t), comp.sum())  # every pass at max(skel, its share of the work)
    print(f"sum of passes {total:.2f} ms (model {pred.sum():.2f}); compute under the skeleton "
          f"(absorbable by moving stages) {slack:.2f} ms; balanced bound {bound:.2f} ms; "
          f"headroom {(pred.sum() - bound) / pred.sum():.1%} of the reverse passes")
    for (k, ms), g, r, s in sorted(zip(rev, G, R, S), key=lambda x: x[0][1]):
        print(f"  {ms:7.3f} ms  gamma {int(g):2d} stages {int(s):2d} relayouts {int(r):2d}  {k}")


if __name__ == "__main__":
    main()

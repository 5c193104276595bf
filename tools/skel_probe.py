#!/usr/bin/env python3
"""Fused-pass time versus where a tile's rows sit in memory (timing probe, not a test).

C2-style layers (Haar q1 on every used qubit, q2 brickwork) restricted to a qubit set, at
n = 28 f32 with permuting passes off, so every pass's tile is the 4 low positions plus the
set's upper 8 qubits as rows.  Prints per-kernel average ms for each set.  Run with the
product library or a timing-only ablation build (QDC_LIB_DIR=build/abl3 QDC_BENCH_ABLATION=1:
load/store skeleton only).

usage: QDC_RQ_PERM=0 python tools/skel_probe.py
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "differentiable-quantum-circuit-cuda_amd"))
import quantum_differentiable_circuit as q  # noqa: E402
from quantum_differentiable_circuit import workloads as W  # noqa: E402

N = int(os.environ.get("SKEL_N", "28"))
SETS = {
    "contig 0..11": list(range(12)),
    "mid 0..3+12..19": [0, 1, 2, 3] + list(range(12, 20)),
    "far 0..3+20..27": [0, 1, 2, 3] + list(range(20, 28)),
    "spread 0..3+{6,9,..27}": [0, 1, 2, 3] + [6, 9, 12, 15, 18, 21, 24, 27],
}


def circuit(qs, layers, rng):
    ins, var = [], []
    for _ in range(layers):
        for p in qs:
            ins.append((W.VAR_Q1, (p,)))
            var.append(W.haar_unitary(rng, 2))
        for start in (0, 1):
            for i in range(start, len(qs) - 1, 2):
                ins.append((W.VAR_Q2, (qs[i + 1], qs[i])))
                var.append(W.haar_unitary(rng, 4))
    for p in qs:
        ins.append((W.DIFF_Q1_DENSITY, (p,)))
    return ins, var


def main():
    rng = np.random.default_rng(1)
    for name, qs in SETS.items():
        ins, var = circuit(qs, 8, rng)
        c = q.circuit_class("f32")(N)
        for kind, pos in ins:
            c._push(kind, *pos)
        vg = [np.ascontiguousarray(g, dtype=np.complex64) for g in var]
        d = c.forward([], vg)
        cots = [np.diag([1.0, -1.0]).astype(np.complex64) for _ in d]
        c.backward(cots, [], vg)
        c.profile(True)
        t0 = time.perf_counter()
        for _ in range(2):
            c.forward([], vg)
            c.backward(cots, [], vg)
        dt = (time.perf_counter() - t0) / 2
        st = c.profile_collect()
        c.profile(False)
        ks = {k: (v["launches"], round(v["total_ms"] / v["launches"], 4)) for k, v in st.items()
              if k.startswith("fused") and v["launches"]}
        print(f"{name:26s} step {dt * 1e3:8.1f} ms  {ks}", flush=True)
        del c


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Host emulation (numpy, complex64 arithmetic) of where the O(1)-memory uncompute error of the
fused runtime comes from, on the runtime's OWN stage schedule (qdc_fusion_schedule: the exact
grouping of gates into stages of the forward and reverse passes).  Config C5's generator
(tests/test_gpu_drift.py), error of the state after forward + uncompute against the complex128
result of the same f32 gate matrices.  Rows:
  per-gate                      the reference's algorithm: U then U^dagger per gate
  fused                         forward stages round(prod U), reverse stages round(prod U^dagger)
  fused fwd, per-gate rev       only the forward fused
  per-gate fwd, fused rev       only the reverse fused
  fused fwd, rev = fwd^dagger   reverse aligned to the forward's rounded stage matrices
  fused, unrounded matrices     stage products applied in complex128, state rounded per stage
usage: python3 tools/drift_emu.py [n] [gates]"""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "differentiable-quantum-circuit-cuda_amd"))

import quantum_differentiable_circuit as q  # noqa: E402
from quantum_differentiable_circuit import workloads as W  # noqa: E402

DT = np.complex128 if os.environ.get("QDC_EMU_DT") == "c128" else np.complex64


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 14
    ng = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
    if len(sys.argv) > 3 and sys.argv[3] == "layered":  # C2's generator, ng layers
        ins, var = W.layered_circuit(n, ng, 24)
    else:
        ins, var = W.deep_random_circuit(n, ng, seed=33)
    instr = [(k, *p) for k, p in ins]
    gm, vi = {}, 0
    for i, (k, p) in enumerate(ins):
        if k in (1, 5, 8):  # VAR_Q2, VAR_Q2_DIAG, VAR_Q1
            gm[i] = (k, p, np.asarray(var[vi]).astype(DT))
            vi += 1

    def apply(psi, u, pos, dt, mat_dt=None):
        k = len(pos)
        t = psi.reshape((2,) * n)
        ax = [n - 1 - p for p in pos]
        t = np.moveaxis(t, ax, list(range(k))).reshape(1 << k, -1)
        t = (u.astype(mat_dt or dt) @ t).astype(dt)
        t = np.moveaxis(t.reshape((2,) * n), list(range(k)), ax)
        return t.reshape(-1)

    def full(k, g):
        g = g.astype(np.complex128)
        return np.diag(g) if k == 5 else g.reshape(2, 2) if k == 8 else g.reshape(4, 4)

    def emb(k, p, m, lo, hi):  # gate matrix in the stage basis 2 bit(hi) + bit(lo)
        if lo == hi:
            return m
        if len(p) == 1:
            return np.kron(m, np.eye(2)) if p[0] == hi else np.kron(np.eye(2), m)
        if p[0] == hi:
            return m
        perm = [0, 2, 1, 3]
        return m[perm][:, perm]

    def stages(mode, dag, split_by=None):
        """stage matrices of the schedule; split_by: gate -> forward stage id, and reverse stages
        are cut where consecutive gates came from different forward stages (aligned stages)"""
        ops, items = q.fusion_schedule(n, instr, mode)
        out = []
        for it in items:
            groups = []
            for st in it["stages"]:
                gi = [ops[j]["instr"] for j in st if ops[j]["instr"] in gm]
                if not gi:
                    continue
                if split_by is None:
                    groups.append(gi)
                    continue
                cur = [gi[0]]
                for g in gi[1:]:
                    if split_by[g] != split_by[cur[-1]]:
                        groups.append(cur)
                        cur = []
                    cur.append(g)
                groups.append(cur)
            for gi in groups:
                qs = sorted({b for i in gi for b in gm[i][1]})
                lo, hi = qs[0], qs[-1]
                a = np.eye(2 if lo == hi else 4, dtype=np.complex128)
                for i in gi:
                    k, p, g = gm[i]
                    m = full(k, g)
                    a = emb(k, p, m.conj().T if dag else m, lo, hi) @ a
                out.append((a, (hi,) if lo == hi else (hi, lo), gi))
        return out

    order = sorted(gm)
    psi0 = np.zeros(1 << n, np.complex128)
    psi0[0] = 1
    ex = psi0.copy()
    for i in order:
        k, p, g = gm[i]
        ex = apply(ex, full(k, g), p, np.complex128)
    for i in reversed(order):
        k, p, g = gm[i]
        ex = apply(ex, full(k, g).conj().T, p, np.complex128)

    def per_gate_fwd(x):
        for i in order:
            k, p, g = gm[i]
            x = apply(x, full(k, g), p, DT)
        return x

    def per_gate_rev(x):
        for i in reversed(order):
            k, p, g = gm[i]
            x = apply(x, full(k, g).conj().T, p, DT)
        return x

    fwd, rev = stages(1, False), stages(2, True)
    fsid = {g: k for k, (_, _, gi) in enumerate(fwd) for g in gi}
    rev_al = stages(2, True, fsid)

    def fused_fwd(x, mat_dt=None):
        for a, p, _ in fwd:
            x = apply(x, a if mat_dt else a.astype(DT), p, DT, mat_dt)
        return x

    def fused_rev(x, mat_dt=None, st=None):
        for a, p, _ in (rev if st is None else st):
            x = apply(x, a if mat_dt else a.astype(DT), p, DT, mat_dt)
        return x

    x0 = psi0.astype(DT)
    rows = {
        "per-gate": per_gate_rev(per_gate_fwd(x0)),
        "fused": fused_rev(fused_fwd(x0)),
        "fused fwd, per-gate rev": per_gate_rev(fused_fwd(x0)),
        "per-gate fwd, fused rev": fused_rev(per_gate_fwd(x0)),
    }
    x = fused_fwd(x0)
    for a, p, _ in reversed(fwd):
        x = apply(x, a.astype(DT).conj().T, p, DT)
    rows["fused fwd, rev = fwd^dagger"] = x
    rows[f"fused, rev stages cut at fwd stages ({len(rev_al)})"] = fused_rev(fused_fwd(x0), st=rev_al)
    x = fused_fwd(x0)
    for a, p, _ in reversed(fwd):
        x = apply(x, np.linalg.inv(a.astype(DT).astype(np.complex128)).astype(DT), p, DT)
    rows["fused fwd, rev = inv(fwd) rounded"] = x
    x = fused_fwd(x0)
    for a, p, _ in reversed(fwd):
        x = apply(x, np.linalg.inv(a.astype(DT).astype(np.complex128)), p, DT, np.complex128)
    rows["fused fwd, rev = inv(fwd) exact"] = x
    rows["fused, unrounded matrices"] = fused_rev(fused_fwd(x0, np.complex128), np.complex128)
    rows["fused fwd rounded, rev unrounded"] = fused_rev(fused_fwd(x0), np.complex128)
    rows["fused fwd unrounded, rev rounded"] = fused_rev(fused_fwd(x0, np.complex128))
    base = np.abs(rows["per-gate"] - ex).max()
    print(f"C5 n={n} {ng} gates: {len(fwd)} forward / {len(rev)} reverse stages "
          f"({len(order) / len(fwd):.2f} / {len(order) / len(rev):.2f} gates per stage)")
    for name, x in rows.items():
        e = np.abs(x - ex).max()
        print(f"{name:30s} uncompute error {e:.3e}  ({e / base:.2f} x per-gate)")


if __name__ == "__main__":
    main()

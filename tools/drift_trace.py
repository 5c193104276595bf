#!/usr/bin/env python3
"""Host emulation of the O(1)-memory uncompute drift on the runtime's OWN program, sharded or
not: the matrices a forward then a backward call apply to the forward state come from the
runtime's dry run (quantum_differentiable_circuit.trace_program -> qdc_trace_program: the exact
stage matrices as uploaded, in execution order, on logical qubits — remaps and permuting
passes are exact permutations, so the logical frame loses nothing).  They are applied to a
complex64 state with complex64 arithmetic, and the error of the state after forward + uncompute
is compared with the reference's gate-by-gate algorithm (U then U^dagger per gate, complex64)
on the same circuit.

usage: python3 tools/drift_trace.py [n] [gates] [worlds, comma-separated] [seed]
Prints per world: stages applied forward / backward, mirrored / own-formed reverse stages,
single-gate items, the uncompute error and its ratio to the per-gate floor."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "differentiable-quantum-circuit-cuda_amd"))

import quantum_differentiable_circuit as q  # noqa: E402
from quantum_differentiable_circuit import workloads as W  # noqa: E402

DT = np.complex64


def apply(psi, u, qs, n, dt=DT):
    """u (2^k x 2^k, row index sum_i bit(qs[i]) 2^(k-1-i)) on logical qubits qs (first = MSB)."""
    k = len(qs)
    t = psi.reshape((2,) * n)
    ax = [n - 1 - p for p in qs]
    t = np.moveaxis(t, ax, list(range(k))).reshape(1 << k, -1)
    t = (u.astype(dt) @ t).astype(dt)
    t = np.moveaxis(t.reshape((2,) * n), list(range(k)), ax)
    return t.reshape(-1)


def run_trace(tr, n, psi0, which=None):
    psi = psi0.astype(DT).copy()
    for op in tr:
        if which is not None and op["dir"] != which:
            continue
        R = int(op["R"])
        u = np.asarray(op["m"][:R * R]).reshape(R, R)
        qs = [int(op["q2"])] if R == 2 else [int(op["q2"]), int(op["q1"])]
        psi = apply(psi, u, qs, n)
    return psi


def per_gate(ins, var, n, psi0):
    """The reference's algorithm (src/circuit.rs:164-429): U per gate forward, U^dagger per gate
    in reverse order (VAR kinds only here: the C5 / C2 generators)."""
    gates = []
    vi = 0
    for k, p in ins:
        if k in (W.VAR_Q1, W.VAR_Q2, W.VAR_Q2_DIAG):
            g = np.asarray(var[vi]).astype(DT)
            vi += 1
            u = np.diag(g) if k == W.VAR_Q2_DIAG else g.reshape(2, 2) if k == W.VAR_Q1 else g.reshape(4, 4)
            gates.append((u, list(p)))
    psi = psi0.astype(DT).copy()
    for u, qs in gates:
        psi = apply(psi, u, qs, n)
    for u, qs in reversed(gates):
        psi = apply(psi, u.conj().T, qs, n)
    return psi


def q1_densities(psi, n, qubits):
    t = psi.astype(np.complex128).reshape((2,) * n)
    out = []
    for qb in qubits:
        a = np.moveaxis(t, n - 1 - qb, 0).reshape(2, -1)
        out.append(a @ a.conj().T)
    return np.concatenate([d.reshape(-1) for d in out])


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 14
    ng = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
    worlds = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "1,2,8").split(",")]
    seed = int(sys.argv[4]) if len(sys.argv) > 4 else 33
    ins, var = W.deep_random_circuit(n, ng, seed=seed)
    instr = [(k, *p) for k, p in ins]
    vg = [np.ascontiguousarray(g, dtype=DT) for g in var]
    cots = [np.diag([1.0, -1.0]).astype(DT) for k, _ in ins if k == W.DIFF_Q1_DENSITY]
    psi0 = np.zeros(1 << n, np.complex128)
    psi0[0] = 1
    ref = per_gate(ins, var, n, psi0)
    dq = [p[0] for k, p in ins if k == W.DIFF_Q1_DENSITY]
    ex = psi0.copy()
    vi = 0
    for k, p in ins:
        if k in (W.VAR_Q1, W.VAR_Q2, W.VAR_Q2_DIAG):
            g = np.asarray(vg[vi]).astype(np.complex128)
            vi += 1
            u = np.diag(g) if k == W.VAR_Q2_DIAG else g.reshape(2, 2) if k == W.VAR_Q1 else g.reshape(4, 4)
            ex = apply(ex, u, list(p), n, np.complex128)
    dex = q1_densities(ex, n, dq)
    rf = psi0.astype(DT)
    for k, p in ins:
        pass
    fw_ref = None
    floor = np.abs(ref - psi0).max()
    floor2 = np.linalg.norm(ref - psi0)
    print(f"n={n} gates={ng} seed={seed}: per-gate (reference) uncompute error {floor:.3e} "
          f"(2-norm {floor2:.3e})")
    for w in worlds:
        tr = q.trace_program(n, instr, [], vg, cots, world=w, precision="f32")
        fw, bw = tr[tr["dir"] == 0], tr[tr["dir"] == 1]
        psi_f = run_trace(tr, n, psi0, which=0)
        derr = np.abs(q1_densities(psi_f, n, dq) - dex).max() / np.abs(dex).max()
        serr = np.abs(psi_f - ex).max() / np.abs(ex).max()
        psi = run_trace(tr, n, psi0)
        err = np.abs(psi - psi0).max()
        err2 = np.linalg.norm(psi - psi0)
        own = int(((bw["single"] == 0) & (bw["mirrored"] == 0)).sum())
        print(f"world {w}: fwd {len(fw)} ops ({int(fw['single'].sum())} single, "
              f"{int((fw['R'] == 4).sum())} two-qubit), bwd {len(bw)} ops "
              f"({int(bw['mirrored'].sum())} mirrored, {own} own-formed, {int(bw['single'].sum())} single), "
              f"state err {serr:.3e}, density err {derr:.3e}, uncompute err {err:.3e} ratio {err / floor:.2f}; 2-norm {err2:.3e} ratio {err2 / floor2:.2f}",
              flush=True)


if __name__ == "__main__":
    main()

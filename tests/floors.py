"""Measured floating-point floors for multi-gate parity tests (test infrastructure).

A fixed tolerance on a circuit either hides real errors (a wrong gradient stage of relative
size 1e-4 passes a 2e-3 bound) or fails deep circuits, because rounding error grows with depth.
Instead, every multi-gate GPU parity test measures the floor of THE SAME circuit: the
reference's own algorithm run in the build's precision — the C restatement of its kernels
(oracle/cpu_ref.c, index rules of src/primitives.cu:176-953) driven by the oracle's
restatement of src/circuit.rs:164-429 (unfused: uncompute, gradient, pull-back per gate,
allocate-conj-gate-add per density) — against the exact result (the einsum oracle in
complex128).  The HIP path must stay within RATIO x that floor (plus ATOL, one rounding of
the working precision, for outputs whose floor is exactly zero).  Every check prints the
measured error, the floor and their ratio.

Norm-relative error throughout: max |a - b| / max |b| over the flattened output group.
"""
from __future__ import annotations

import numpy as np

from oracle import oracle as O
from oracle.cref import CRefOps

RATIO = 4.0
ATOL = {"f32": 2.4e-7, "f64": 1e-15}
DT = {"f32": np.complex64, "f64": np.complex128}


def flat(xs):
    if isinstance(xs, np.ndarray):
        return xs.reshape(-1)
    return np.concatenate([np.asarray(x).reshape(-1) for x in xs]) if len(xs) else np.zeros(0)


def l2rel(a, b):
    """2-norm relative error ||a - b|| / ||b||: an aggregate over every element, so one circuit's
    value is a stable statistic of its rounding (the max-norm of normrel is the extreme of 2^n
    random-walk endpoints and varies ~0.3-2x between realizations, tools/drift_trace.py)."""
    a, b = flat(a).astype(np.complex128), flat(b).astype(np.complex128)
    den = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / den) if den > 0 else float(np.linalg.norm(a - b))


def normrel(a, b):
    a, b = flat(a).astype(np.complex128), flat(b).astype(np.complex128)
    den = np.abs(b).max() if b.size else 0.0
    return float(np.abs(a - b).max() / den) if den > 0 else float(np.abs(a - b).max())


def sigma_z_cots(dens, dt):
    """Cotangents of sum Re tr(rho Z x Z...) (diagonal +-1, Hermitian)."""
    return [np.ascontiguousarray(np.diag([1.0, -1.0] if d.shape == (2, 2)
                                         else [1.0, -1.0, -1.0, 1.0]).astype(dt)) for d in dens]


def tsallis_cots(dens, dt):
    """conj of the JAX cotangents of the mean Tsallis-2 entropy (test_autodiff.py:87-92,
    circuit.py:193), from complex128 densities."""
    _, cots = O.tsallis_loss_and_cotangents([np.asarray(d, np.complex128) for d in dens])
    return [np.ascontiguousarray(x.conj(), dtype=dt) for x in cots]


def oracle_outputs(n, ins, const, var, psi0=None, cots=None, ops=None, run=True):
    """run / forward densities, gradients and the states of one call sequence
    (run, forward, backward) on the oracle circuit with op table `ops` (None: complex128
    einsum).  `cots`: the cotangents to feed backward (a callable of the forward densities,
    or a list)."""
    o = O.OracleCircuit(n, np.complex128, ops=ops or O.EinsumOps)
    for kind, pos in ins:
        o.add(kind, *pos)
    if psi0 is not None:
        o.set_state_from_vector(psi0)
    out = {}
    if run:
        out["run"] = o.run(const, var)
    out["forward"] = o.forward(const, var)
    out["state"] = np.asarray(o.state, np.complex128).copy()
    if cots is not None:
        cl = cots(out["forward"]) if callable(cots) else cots
        out["cots"] = cl
        out["grads"] = o.backward(cl, const, var)
        out["uncomputed"] = np.asarray(o.state, np.complex128).copy()
        if o.bwd is not None:
            out["bwd"] = np.asarray(o.bwd, np.complex128).copy()
    return out


class Floor:
    """The exact outputs of a circuit and the floor of each output group."""

    def __init__(self, prec, n, ins, const, var, psi0=None, cots=sigma_z_cots, run=True,
                 exact_ops=None):
        """exact_ops: the op table of the exact result (None: the complex128 einsum oracle;
        CRefOps("f64") at sizes where einsum is too slow — then `prec` must be "f32", whose
        floor is ~1e9 times the f64 restatement's own rounding)."""
        self.prec = prec
        dt = DT[prec]
        self.const = [np.ascontiguousarray(g, dtype=dt) for g in const]
        self.var = [np.ascontiguousarray(g, dtype=dt) for g in var]
        self.psi0 = None if psi0 is None else np.ascontiguousarray(psi0, dtype=dt)
        # exact result of the build-precision inputs; the cotangents are computed once (from
        # the exact forward densities) and fed to every run
        exact = oracle_outputs(n, ins, self.const, self.var, self.psi0,
                               (lambda d: cots(d, dt)) if cots is not None else None, ops=exact_ops,
                               run=run)
        self.cots = exact.get("cots")
        ref = oracle_outputs(n, ins, self.const, self.var, self.psi0, self.cots, ops=CRefOps(prec),
                             run=run)
        self.exact = exact
        self.floor = {k: normrel(ref[k], exact[k]) for k in exact if k != "cots"}
        self.floor_l2 = {k: l2rel(ref[k], exact[k]) for k in exact if k != "cots"}

    def check(self, key, got, what="", ratio=RATIO):
        err = normrel(got, self.exact[key])
        fl = self.floor[key]
        bound = ratio * fl + ATOL[self.prec]
        # which term admits the result: ratio x floor alone, or only with the one-rounding ATOL
        binding = "floor" if err <= ratio * fl else "ATOL"
        print(f"[floor] {what}{key}: err {err:.3e}  floor {fl:.3e}  "
              f"ratio {err / fl if fl > 0 else float('inf'):.2f}  bound {bound:.3e}  "
              f"passes-by {binding}")
        assert err <= bound, f"{what}{key}: error {err:.3e} > {ratio} x floor {fl:.3e} + atol"
        return err


    def check_l2(self, key, got, what="", ratio=RATIO):
        """As check, in the 2-norm: the stable aggregate of the same rounding (state outputs)."""
        err = l2rel(got, self.exact[key])
        fl = self.floor_l2[key]
        bound = ratio * fl + ATOL[self.prec]
        binding = "floor" if err <= ratio * fl else "ATOL"
        print(f"[floor-l2] {what}{key}: err {err:.3e}  floor {fl:.3e}  "
              f"ratio {err / fl if fl > 0 else float('inf'):.2f}  bound {bound:.3e}  "
              f"passes-by {binding}")
        assert err <= bound, f"{what}{key}: 2-norm error {err:.3e} > {ratio} x floor {fl:.3e} + atol"
        return err


def check_pair(prec, a, b, floor_value, what, ratio=2 * RATIO):
    """Two HIP results of the same circuit (e.g. sharded vs unsharded, fused vs unfused): each is
    within RATIO x floor of the exact result, so they differ by at most 2 RATIO x floor."""
    err = normrel(a, b)
    bound = ratio * floor_value + 2 * ATOL[prec]
    binding = "floor" if err <= ratio * floor_value else "ATOL"
    print(f"[floor] {what}: diff {err:.3e}  floor {floor_value:.3e}  bound {bound:.3e}  "
          f"passes-by {binding}")
    assert err <= bound, f"{what}: difference {err:.3e} > {ratio} x floor {floor_value:.3e}"
    return err

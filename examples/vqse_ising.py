#!/usr/bin/env python3
"""VQSE of the critical transverse-field Ising chain on the HIP path — the reference's
example_vqse_ising.py (config C3 of SURVEY.md §8 d) without JAX: qdc.AutoGradCircuit's
VJPFunction supplies the circuit's pullback, workloads.vqse_loss_and_grad chains it to the real
parameters, scipy's L-BFGS-B optimises.

  python examples/vqse_ising.py [--qubits 26] [--layers 26] [--iters 300] [--precision f64]

The example's parameters: n = 26, 26 layers, |+>^n initial state, field 1 (the phase
transition), L-BFGS-B up to 300 iterations; PRNG seed 42 (numpy's, JAX being absent)."""
import argparse
import sys
import time
from pathlib import Path

import numpy as np
from scipy.optimize import minimize

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "differentiable-quantum-circuit-cuda_amd"))

from qdc import AutoGradCircuit  # noqa: E402
from quantum_differentiable_circuit import workloads as W  # noqa: E402


def build(n, layers, precision):
    c = AutoGradCircuit(n, precision=precision)
    state = np.ones(1 << n, dtype=c.dtype) / np.sqrt(1 << n)
    c.set_state_from_vector(state)
    for kind, pos in W.vqse_ising(n, layers):
        if kind == W.VAR_Q2_DIAG:
            c.add_q2_var_gate_diag(*pos)
        elif kind == W.VAR_Q1:
            c.add_q1_var_gate(*pos)
        else:
            c.get_q2_dens_op_with_grad(*pos)
    _, fwd_circ = c.build()
    return lambda gates: fwd_circ.vjp(gates, [])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--qubits", type=int, default=26)
    ap.add_argument("--layers", type=int, default=26)
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--precision", default="f64", choices=["f32", "f64"])
    ap.add_argument("--seed", type=int, default=42)
    args = ap.parse_args()
    n = args.qubits
    fwd_vjp = build(n, args.layers, args.precision)
    h = W.tfim_term(1.0)
    params = np.random.default_rng(args.seed).normal(size=2 * args.layers)
    calls = [0]

    def loss_val_and_grad(p):
        calls[0] += 1
        return W.vqse_loss_and_grad(fwd_vjp, p, n, h)

    start = time.time()
    result = minimize(loss_val_and_grad, params, method="L-BFGS-B", jac=True,
                      options={"maxiter": args.iters})
    end = time.time()
    exact_e = -2 * (1 / np.sin(np.pi / (2 * n)))
    print(f"Exact energy: {exact_e}")
    print(f"Found energy: {result.fun}")
    print(f"Relative error: {abs(result.fun - exact_e) / abs(exact_e)}")
    print(f"Number of loss value and gradient calls: {calls[0]}")
    print(f"Time per loss value and gradient call: {(end - start) / calls[0]}")


if __name__ == "__main__":
    main()

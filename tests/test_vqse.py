"""Config C3's host logic (example_vqse_ising.py without JAX): the VQSE workload, its
parameter-to-gate map and the chain rule of workloads.vqse_loss_and_grad, checked on the oracle
backend against central finite differences (CPU).  The HIP-backed runs are in
tests/test_gpu_vqse.py."""
import numpy as np

from oracle import oracle as O
from quantum_differentiable_circuit import workloads as W


def oracle_vjp(n, layers):
    o = O.OracleCircuit(n, np.complex128)
    for kind, pos in W.vqse_ising(n, layers):
        o.add(kind, *pos)
    o.set_state_from_vector(np.ones(1 << n, dtype=np.complex128) / np.sqrt(1 << n))

    def fwd_vjp(gates):
        dens = o.forward([], gates)
        # qdc's custom_vjp backward conjugates the density cotangents (circuit.py:193)
        return dens, lambda cots: (o.backward([np.conj(c) for c in cots], [], gates), None)
    return fwd_vjp


def test_vqse_structure():
    ins = W.vqse_ising(26, 26)
    assert len(ins) == 26 * 52 + 26
    assert sum(k == W.DIFF_Q2_DENSITY for k, _ in ins) == 26
    assert len(W.vqse_gates(np.zeros(52), 26)) == 26 * 52


def test_vqse_gradient_matches_finite_differences():
    n, layers = 6, 3
    fwd_vjp = oracle_vjp(n, layers)
    h = W.tfim_term(1.0)
    p = np.random.default_rng(42).normal(size=2 * layers)
    e, g = W.vqse_loss_and_grad(fwd_vjp, p, n, h)
    eps = 1e-5
    fd = np.array([(W.vqse_loss_and_grad(fwd_vjp, p + eps * u, n, h)[0] -
                    W.vqse_loss_and_grad(fwd_vjp, p - eps * u, n, h)[0]) / (2 * eps)
                   for u in np.eye(len(p))])
    assert np.abs(fd - g).max() <= 1e-7 * max(1.0, np.abs(g).max()), (fd, g)
    # |+>^n at zero angles: every X-term density gives <X> = 1, so E = -n(1) - n field/2 * 2
    e0, _ = W.vqse_loss_and_grad(fwd_vjp, np.zeros(2 * layers), n, h)
    assert abs(e0 - (-n * 1.0)) < 1e-12

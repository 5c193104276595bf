"""Config C3 (SURVEY.md §8 d): VQSE on the critical transverse-field Ising chain
(example_vqse_ising.py) through qdc.AutoGradCircuit on the HIP path.

- energy and parameter gradient vs the oracle backend at n = 10 (f32, f64);
- L-BFGS-B at n = 8 reaches the exact critical energy -2/sin(pi/2n) (example:127);
- full size, n = 26 f64, 26 layers (1352 gates, 26 DiffQ2Density): the finite-difference
  identity along a random parameter direction and the variational bound E >= E_exact
  (size-independent properties; the oracle would need minutes per call there)."""
import sys
from pathlib import Path

import numpy as np
import pytest
from scipy.optimize import minimize

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "examples"))

from quantum_differentiable_circuit import workloads as W  # noqa: E402
from test_vqse import oracle_vjp  # noqa: E402

pytestmark = pytest.mark.gpu


def hip_vjp(n, layers, precision):
    import vqse_ising
    return vqse_ising.build(n, layers, precision)


@pytest.mark.parametrize("prec,tol", [("f32", 2e-5), ("f64", 1e-11)])
def test_vqse_energy_and_gradient_vs_oracle(prec, tol):
    n, layers = 10, 4
    h = W.tfim_term(1.0)
    p = np.random.default_rng(42).normal(size=2 * layers)
    e, g = W.vqse_loss_and_grad(hip_vjp(n, layers, prec), p, n, h)
    e0, g0 = W.vqse_loss_and_grad(oracle_vjp(n, layers), p, n, h)
    assert abs(e - e0) <= tol * abs(e0)
    assert np.abs(g - g0).max() <= tol * 10 * np.abs(g0).max()


def test_vqse_lbfgs_reaches_exact_energy():
    n, layers = 8, 4
    f = hip_vjp(n, layers, "f64")
    h = W.tfim_term(1.0)
    p = np.random.default_rng(42).normal(size=2 * layers)
    r = minimize(lambda x: W.vqse_loss_and_grad(f, x, n, h), p, method="L-BFGS-B", jac=True,
                 options={"maxiter": 150})
    exact = -2 / np.sin(np.pi / (2 * n))
    assert abs(r.fun - exact) <= 1e-6 * abs(exact), (r.fun, exact)


def test_vqse_full_size_fd_identity_and_variational_bound():
    n, layers = 26, 26
    f = hip_vjp(n, layers, "f64")
    h = W.tfim_term(1.0)
    rng = np.random.default_rng(42)
    p = rng.normal(size=2 * layers)
    d = rng.normal(size=2 * layers)
    d /= np.linalg.norm(d)
    e, g = W.vqse_loss_and_grad(f, p, n, h)
    eps = 1e-4
    ep = W.vqse_loss_and_grad(f, p + eps * d, n, h)[0]
    em = W.vqse_loss_and_grad(f, p - eps * d, n, h)[0]
    fd = (ep - em) / (2 * eps)
    assert abs(fd - g @ d) <= 1e-6 * max(1.0, np.abs(g).max()), (fd, g @ d)
    exact = -2 / np.sin(np.pi / (2 * n))
    for x in (e, ep, em):
        assert x >= exact - 1e-9 and x <= n * 2.0

"""Config C3 (SURVEY.md §8 d): VQSE on the critical transverse-field Ising chain
(example_vqse_ising.py) through qdc.AutoGradCircuit on the HIP path.

- energy and parameter gradient vs the oracle backend at n = 10 (f32, f64), each within 4x the
  measured floor of the reference's own algorithm in the build's precision (the C restatement
  of its kernels, oracle/cpu_ref.c, driven by the oracle's circuit.rs order: tests/floors.py);
- L-BFGS-B at n = 8 reaches the exact critical energy -2/sin(pi/2n) (example:127);
- full size, n = 26, 26 layers (1352 gates, 26 DiffQ2Density) in both precisions — f64 as
  BASELINE.json's config names it, complex64 as the example itself runs
  (example_vqse_ising.py:58,87-89): the finite-difference identity along a random parameter
  direction and the variational bound E >= E_exact (size-independent properties; the oracle
  would need minutes per call there)."""
import sys
from pathlib import Path

import numpy as np
import pytest
from scipy.optimize import minimize

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "examples"))

import floors as F  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle.cref import CRefOps  # noqa: E402
from quantum_differentiable_circuit import workloads as W  # noqa: E402
from test_vqse import oracle_vjp  # noqa: E402

pytestmark = pytest.mark.gpu


def hip_vjp(n, layers, precision):
    import vqse_ising
    return vqse_ising.build(n, layers, precision)


def _vjp_in(n, layers, prec, ops):
    """The oracle's VQSE pullback on op table `ops` with the build-precision inputs (gates,
    |+>^n, cotangents rounded to `prec` first): ops = EinsumOps gives their exact result,
    CRefOps(prec) the reference's algorithm in that precision."""
    dt = F.DT[prec]
    o = O.OracleCircuit(n, np.complex128, ops=ops)
    for kind, pos in W.vqse_ising(n, layers):
        o.add(kind, *pos)
    o.set_state_from_vector((np.ones(1 << n) / np.sqrt(1 << n)).astype(dt))

    def fwd_vjp(gates):
        g = [np.ascontiguousarray(x, dtype=dt) for x in gates]
        dens = o.forward([], g)
        return dens, lambda cots: (o.backward([np.conj(c).astype(dt) for c in cots], [], g), None)
    return fwd_vjp


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_vqse_energy_and_gradient_vs_oracle(prec):
    n, layers = 10, 4
    h = W.tfim_term(1.0)
    p = np.random.default_rng(42).normal(size=2 * layers)
    e, g = W.vqse_loss_and_grad(hip_vjp(n, layers, prec), p, n, h)
    e0, g0 = W.vqse_loss_and_grad(_vjp_in(n, layers, prec, O.EinsumOps), p, n, h)
    er, gr = W.vqse_loss_and_grad(_vjp_in(n, layers, prec, CRefOps(prec)), p, n, h)
    what = f"C3 VQSE n={n} {prec} "
    for key, got, ref, ex in (("energy", e, er, e0), ("grad", g, gr, g0)):
        err, fl = F.normrel(np.atleast_1d(got), np.atleast_1d(ex)), F.normrel(np.atleast_1d(ref), np.atleast_1d(ex))
        bound = F.RATIO * fl + F.ATOL[prec]
        print(f"[floor] {what}{key}: err {err:.3e}  floor {fl:.3e}  "
              f"ratio {err / fl if fl > 0 else float('inf'):.2f}  bound {bound:.3e}  "
              f"passes-by {'floor' if err <= F.RATIO * fl else 'ATOL'}")
        assert err <= bound, (key, err, fl)
    # and the complex128 oracle of the unrounded inputs (the reference's own test metric)
    e1, _ = W.vqse_loss_and_grad(oracle_vjp(n, layers), p, n, h)
    tol = 2e-5 if prec == "f32" else 1e-11
    assert abs(e - e1) <= tol * abs(e1)


def test_vqse_lbfgs_reaches_exact_energy():
    n, layers = 8, 4
    f = hip_vjp(n, layers, "f64")
    h = W.tfim_term(1.0)
    p = np.random.default_rng(42).normal(size=2 * layers)
    r = minimize(lambda x: W.vqse_loss_and_grad(f, x, n, h), p, method="L-BFGS-B", jac=True,
                 options={"maxiter": 150})
    exact = -2 / np.sin(np.pi / (2 * n))
    assert abs(r.fun - exact) <= 1e-6 * abs(exact), (r.fun, exact)


# Finite-difference step and tolerance per precision.  f64: eps 1e-4 (truncation ~eps^2 times
# the third derivative), 1e-6 of max(1, |g|).  f32: the energy sums 26 densities of 2^26
# complex64 amplitudes, so its rounding is ~1e-6 of |E| ~ 33 and a central difference with
# eps 1e-2 carries ~1e-6 * 33 / 1e-2 ~ 3e-3 of it, truncation ~1e-3: 1e-2 admits both.
FD = {"f64": (1e-4, 1e-6), "f32": (1e-2, 1e-2)}


@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_vqse_full_size_fd_identity_and_variational_bound(prec):
    n, layers = 26, 26
    f = hip_vjp(n, layers, prec)
    h = W.tfim_term(1.0)
    rng = np.random.default_rng(42)
    p = rng.normal(size=2 * layers)
    d = rng.normal(size=2 * layers)
    d /= np.linalg.norm(d)
    e, g = W.vqse_loss_and_grad(f, p, n, h)
    eps, tol = FD[prec]
    ep = W.vqse_loss_and_grad(f, p + eps * d, n, h)[0]
    em = W.vqse_loss_and_grad(f, p - eps * d, n, h)[0]
    fd = (ep - em) / (2 * eps)
    scale = max(1.0, np.abs(g).max())
    print(f"[fd] C3 VQSE n={n} {prec}: E {e:.7f}  finite difference {fd:.6e}  analytic {g @ d:.6e}"
          f"  |diff| / max(1, |g|) {abs(fd - g @ d) / scale:.2e}  bound {tol:.0e}")
    assert abs(fd - g @ d) <= tol * scale, (fd, g @ d)
    exact = -2 / np.sin(np.pi / (2 * n))
    slack = 1e-9 if prec == "f64" else 1e-4 * abs(exact)  # (f32: the energy's own rounding)
    for x in (e, ep, em):
        assert x >= exact - slack and x <= n * 2.0


def test_vqse_full_size_f32_vs_f64():
    """The complex64 run against the complex128 run of the same n = 26 call (energy and the 52
    real-parameter gradients): the f32 rounding of a 1352-gate call, ~1e-6 relative."""
    n, layers = 26, 26
    h = W.tfim_term(1.0)
    p = np.random.default_rng(7).normal(size=2 * layers)
    e64, g64 = W.vqse_loss_and_grad(hip_vjp(n, layers, "f64"), p, n, h)
    e32, g32 = W.vqse_loss_and_grad(hip_vjp(n, layers, "f32"), p, n, h)
    de, dg = abs(e32 - e64) / abs(e64), np.abs(g32 - g64).max() / np.abs(g64).max()
    print(f"[f32-vs-f64] C3 VQSE n={n}: energy {de:.2e}, gradient {dg:.2e} (norm-relative)")
    assert de <= 2e-5 and dg <= 2e-4, (de, dg)

"""Mirrored reverse sweeps (QDC_MIRROR) on the GPU against the oracle floors.

With QDC_MIRROR the forward is scheduled so that its fused passes, run in reverse, are the
backward's passes, and each backward stage uncomputes with exactly the adjoint of the stage
matrix the forward applied (qdc_circuit.hpp mirror_schedule / build_program).  The uncompute then
drifts like the reference's gate-by-gate U, U^dagger pairs (src/circuit.rs:266-429) instead of
accumulating the rounding of independently formed forward and reverse stage products.
QDC_MIRROR=2 makes a backward that cannot mirror its forward an error, so these tests prove the
mirrored schedule ran.  Every output must stay within 4x the floor of the reference's own
algorithm (tests/floors.py); the uncomputed state is the output the mirror exists for.
"""
import numpy as np
import pytest

import floors as F
from oracle import oracle as O
from quantum_differentiable_circuit import workloads as W

pytestmark = pytest.mark.gpu


def build(prec, n, ins):
    import quantum_differentiable_circuit as q
    c = q.circuit_class(prec)(n)
    for kind, pos in ins:
        c._push(kind, *pos)
    return c


@pytest.fixture
def strict_mirror(monkeypatch):
    monkeypatch.setenv("QDC_MIRROR", "2")


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_mirror_c5_depth_10k_gates(strict_mirror, prec):
    n = 14
    ins, var = W.deep_random_circuit(n, 10000, seed=33)
    fl = F.Floor(prec, n, ins, [], var, run=False)
    c = build(prec, n, ins)
    what = f"mirror C5 n={n} 10k {prec} "
    fl.check("forward", c.forward([], fl.var), what)
    fl.check("state", c.get_state(0), what)
    fl.check("grads", c.backward(fl.cots, [], fl.var), what)
    fl.check("uncomputed", c.get_state(0), what)
    fl.check("bwd", c.get_state(2), what)


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_mirror_layered_c2(strict_mirror, prec):
    n = 12
    ins, var = O.layered_circuit(n, layers=4, seed=24)
    fl = F.Floor(prec, n, ins, [], var, run=False)
    c = build(prec, n, ins)
    what = f"mirror C2 n={n} {prec} "
    fl.check("forward", c.forward([], fl.var), what)
    fl.check("grads", c.backward(fl.cots, [], fl.var), what)
    fl.check("uncomputed", c.get_state(0), what)


@pytest.mark.parametrize("prec", ["f32", "f64"])
@pytest.mark.parametrize("n", [12, 17])
def test_mirror_random_every_kind(strict_mirror, prec, n):
    """Every gate kind (NonU kinds uncompute with the inverse, not the mirrored adjoint),
    perturbed non-unitary variable gates (inexact ordering rules) and densities between the
    passes, from a random initial state, Tsallis cotangents."""
    ins, const, var = O.random_circuit(n, 160, seed=100 + n, density_every=40)
    rng = np.random.default_rng(n)
    var = [g + 1e-3 * (rng.standard_normal(g.shape) + 1j * rng.standard_normal(g.shape))
           for g in var]
    psi0 = O.random_state(np.random.default_rng(n), n)
    fl = F.Floor(prec, n, ins, const, var, psi0=psi0, cots=F.tsallis_cots, run=False)
    c = build(prec, n, ins)
    c.set_state_from_vector(fl.psi0)
    what = f"mirror random n={n} {prec} "
    fl.check("forward", c.forward(fl.const, fl.var), what)
    fl.check("grads", c.backward(fl.cots, fl.const, fl.var), what)
    fl.check("uncomputed", c.get_state(0), what)
    fl.check("bwd", c.get_state(2), what)


def test_mirror_needs_the_forwards_gates(strict_mirror):
    """A backward with gates other than its forward's cannot mirror it (QDC_MIRROR=2: error;
    QDC_MIRROR=1 schedules the backward itself)."""
    n = 12
    ins, var = O.layered_circuit(n, layers=2, seed=5)
    fl = F.Floor("f32", n, ins, [], var, run=False)
    c = build("f32", n, ins)
    c.forward([], fl.var)
    other = [(g * np.exp(0.1j)).astype(np.complex64) for g in fl.var]
    with pytest.raises(BaseException, match="mirror"):  # PanicException (as the reference's)
        c.backward(fl.cots, [], other)

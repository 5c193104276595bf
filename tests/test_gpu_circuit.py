"""GPU parity of the circuit runtime (Circuit.run / forward / backward, AutoGradCircuit)
against the oracle's restatement of src/circuit.rs:164-429.

Tolerances: single ops at the north_star's 1e-5 (f32) / 1e-12 (f64), norm-relative
(max |a-b| / max |b|; SURVEY.md §8c: per-element relative error is ill-conditioned for
cancelling sums); multi-gate circuits within 4x the measured floor of the reference's own
algorithm on the same circuit (tests/floors.py); the FD identity at the reference's own 1e-9
(test_autodiff.py:165).
"""
import numpy as np
import pytest

import floors as F
from oracle import oracle as O

pytestmark = pytest.mark.gpu

DT = {"f32": np.complex64, "f64": np.complex128}
TOL = {"f32": 1e-5, "f64": 1e-12}


def close(a, b, tol):
    a, b = np.asarray(a).reshape(-1), np.asarray(b).reshape(-1)
    scale = max(np.abs(b).max(), 1e-300)
    err = np.abs(a - b).max() / scale
    assert err <= tol, f"norm-relative error {err:.3e} > {tol:.1e}"
    return err


def make_pair(prec, n, ins):
    import quantum_differentiable_circuit as q
    c = q.circuit_class(prec)(n)
    o = O.OracleCircuit(n, DT[prec])
    for kind, pos in ins:
        c._push(kind, *pos)
        o.add(kind, *pos)
    return c, o


def cast(gates, prec):
    return [np.ascontiguousarray(g, dtype=DT[prec]) for g in gates]


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_autodiff_structure_parity(prec):
    """Every instruction kind (the test_autodiff.py:49-81 layer) through run/forward/backward,
    within 4x the measured floor of the reference's algorithm (tests/floors.py)."""
    import quantum_differentiable_circuit as q
    n, layers = 9, 3
    ins, const, var, _ = O.autodiff_circuit(n, layers, seed=42)
    psi0 = O.random_state(np.random.default_rng(0), n)
    fl = F.Floor(prec, n, ins, const, var, psi0=psi0, cots=F.tsallis_cots)
    c = q.circuit_class(prec)(n)
    for kind, pos in ins:
        c._push(kind, *pos)
    c.set_state_from_vector(fl.psi0)
    what = f"autodiff n={n} {prec} "
    fl.check("run", c.run(fl.const, fl.var), what)
    got = c.forward(fl.const, fl.var)
    assert len(got) == len(fl.exact["forward"])
    fl.check("forward", got, what)
    fl.check("state", c.get_state(0), what)
    g = c.backward(fl.cots, fl.const, fl.var)
    assert [x.shape for x in g] == [x.shape for x in fl.exact["grads"]]
    fl.check("grads", g, what)
    fl.check("uncomputed", c.get_state(0), what)
    fl.check("bwd", c.get_state(2), what)


def test_finite_difference_identity():
    """test_autodiff.py:121-165 verbatim in structure: n = 15, 10 layers, every gate kind,
    8th-order central differences with eta = 1e-6 along a random complex direction, compared
    with sum Re(g . p) at relative 1e-9 (f64)."""
    from qdc import AutoGradCircuit
    n, layers, eta = 15, 10, 1e-6
    ins, const, var, pert = O.autodiff_circuit(n, layers, seed=42)
    c = AutoGradCircuit(n, precision="f64")
    psi0 = np.zeros(1 << n, np.complex128)
    psi0[0] = 1
    c.set_state_from_vector(psi0)
    for kind, pos in ins:
        c.circuit._push(kind, *pos)
    _, fwd_circ = c.build()

    def tsallis(v):
        dens = fwd_circ(v, const)
        return O.tsallis_loss_and_cotangents(dens)[0]

    coeff = {-4: 1 / 280, -3: -4 / 105, -2: 1 / 5, -1: -4 / 5,
             1: 4 / 5, 2: -1 / 5, 3: 4 / 105, 4: -1 / 280}
    ds_fd = sum(w * tsallis([g + k * eta * p for g, p in zip(var, pert)])
                for k, w in coeff.items()) / eta
    dens, pullback = fwd_circ.vjp(var, const)
    _, cots = O.tsallis_loss_and_cotangents(dens)
    grads, none = pullback(cots)
    assert none is None
    ds = sum(np.tensordot(g, p, axes=1).real for g, p in zip(grads, pert))
    assert abs(ds - ds_fd) / min(abs(ds), abs(ds_fd)) < 1e-9


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_ghz_circuit(prec):
    """test_ghz.py:16-60 with the qdc wiring (numpy VJP driver in place of JAX)."""
    from qdc import AutoGradCircuit
    from quantum_differentiable_circuit.common_gates import get_cnot, get_hadamard
    n = 21
    cnot, h = get_cnot(prec), get_hadamard(prec)  # common_gates.rs:19-34
    c = AutoGradCircuit(n, precision=prec)
    c.add_q1_const_gate(0)
    for i in range(n - 1):
        c.get_q2_dens_op_with_grad(i, i + 1)
    for i in range(n):
        c.get_q1_dens_op_with_grad(i)
    for i in range(n - 1):
        c.add_q2_const_gate(i, i + 1)
    for i in range(n):
        c.get_q1_dens_op(i)
    for i in range(n - 1):
        c.get_q2_dens_op(i, i + 1)
    simple_run, autodiff_run = c.build()
    alld = simple_run([], [h] + (n - 1) * [cnot])
    add = autodiff_run([], [h] + (n - 1) * [cnot])
    assert len(alld) == 2 * n + 2 * (n - 1)
    assert len(add) == n + (n - 1)
    for lhs, rhs in zip(alld[:n + (n - 1)], add):
        assert np.allclose(lhs, rhs)
    first_psi = np.tensordot(np.array([1, 1]) / np.sqrt(2), np.array([1., 0.]), axes=0).reshape(4)
    assert np.allclose(np.outer(first_psi, first_psi.conj()), alld[0])
    second = np.zeros((4, 4))
    second[0, 0] = 1
    for d in alld[1:n - 1]:
        assert np.allclose(d, second)
    assert np.allclose(np.full((2, 2), .5), alld[n - 1])
    for d in alld[n:2 * n - 1]:
        assert np.allclose(d, np.array([[1, 0], [0, 0]]))
    for d in alld[2 * n - 1:3 * n - 1]:
        assert np.allclose(d, np.eye(2) / 2)
    two = np.zeros((4, 4))
    two[0, 0] = two[3, 3] = .5
    for d in alld[3 * n - 1:]:
        assert np.allclose(d, two)


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_layered_c2_parity(prec):
    """Config C2's generator at n = 12 against the oracle (floors)."""
    import quantum_differentiable_circuit as q
    n = 12
    ins, var = O.layered_circuit(n, layers=4, seed=24)
    fl = F.Floor(prec, n, ins, [], var, run=False)
    c = q.circuit_class(prec)(n)
    for kind, pos in ins:
        c._push(kind, *pos)
    fl.check("forward", c.forward([], fl.var), f"C2 n={n} {prec} ")
    fl.check("grads", c.backward(fl.cots, [], fl.var), f"C2 n={n} {prec} ")
    fl.check("uncomputed", c.get_state(0), f"C2 n={n} {prec} ")


@pytest.mark.timeout(900)
def test_layered_c2_n24_f32_vs_f64_restatement():
    """BASELINE config 2 at its stated size: C2's generator at n = 24, f32, forward + backward
    on the GPU, against the reference algorithm in complex128 (the C restatement of its kernels,
    CRefOps("f64"), driven in circuit.rs order — exact to ~1e-15 here, far below the f32
    floor).  The floor is the same restatement in f32.  4 layers (220 gates, 24 densities): the
    two host runs of the reference algorithm take about a minute on the box's cores."""
    import quantum_differentiable_circuit as q
    from oracle.cref import CRefOps
    n = 24
    ins, var = O.layered_circuit(n, layers=4, seed=24)
    fl = F.Floor("f32", n, ins, [], var, run=False, exact_ops=CRefOps("f64"))
    c = q.circuit_class("f32")(n)
    for kind, pos in ins:
        c._push(kind, *pos)
    fl.check("forward", c.forward([], fl.var), f"C2 n={n} f32 ")
    fl.check("grads", c.backward(fl.cots, [], fl.var), f"C2 n={n} f32 ")
    fl.check("uncomputed", c.get_state(0), f"C2 n={n} f32 ")
    fl.check("bwd", c.get_state(2), f"C2 n={n} f32 ")


def test_uncompute_roundtrip_large():
    """Size-independent property at a large size (n = 26, f32): the O(1)-memory reverse sweep
    returns the forward state to the initial state, and gradients of unitary circuits satisfy
    sum_k Re tr(G_k^T ... ) structure checks are replaced by the forward/backward invariants:
    norm conservation and psi0 recovery."""
    import quantum_differentiable_circuit as q
    n = 26
    ins, var = O.layered_circuit(n, layers=2, seed=26)
    c = q.circuit_class("f32")(n)
    for kind, pos in ins:
        c._push(kind, *pos)
    vg = cast(var, "f32")
    dens = c.forward([], vg)
    for d in dens:
        assert abs(np.trace(d) - 1) < 1e-4
        assert np.allclose(d, d.conj().T, atol=1e-5)
    cots = [np.ascontiguousarray(np.diag([1.0, -1.0]).astype(np.complex64)) for _ in dens]
    grads = c.backward(cots, [], vg)
    assert all(np.isfinite(g).all() for g in grads)
    psi = c.get_state(0)
    assert abs(psi[0] - 1) < 1e-4 and np.abs(psi[1:]).max() < 1e-4


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_panics(prec):
    import quantum_differentiable_circuit as q
    C = q.circuit_class(prec)
    g4 = np.eye(2, dtype=DT[prec]).reshape(-1)
    g16 = np.eye(4, dtype=DT[prec]).reshape(-1)
    c = C(3)
    with pytest.raises(q.PanicException, match="The circuit is empty."):
        c.run([], [])
    c.add_q1_const_gate(0)
    with pytest.raises(q.PanicException, match="The number of constant gates is less than required."):
        c.run([], [])
    with pytest.raises(q.PanicException, match="Number of constant gates is more than required."):
        c.run([g4, g4], [])
    with pytest.raises(q.PanicException, match="Number of variable gates is more than required."):
        c.run([g4], [g4])
    with pytest.raises(q.PanicException, match="Incorrect len of the gate's buffer."):
        c.run([g16], [])
    c.add_q2_var_gate_diag(1, 2)
    # circuit.rs:198 reports the constant-gate message for a missing VarQ2GateDiag gate
    with pytest.raises(q.PanicException, match="The number of constant gates is less than required."):
        c.forward([g4], [])
    c.add_q2_var_gate(2, 2)
    with pytest.raises(q.PanicException, match="pos1 and pos2 must be different."):
        c.forward([g4], [g4, g16])
    d = C(3)
    d.add_q1_var_gate(5)
    with pytest.raises(q.PanicException, match="pos is out of the bound."):
        d.forward([], [g4])
    e = C(3)
    e.add_q1_var_gate(0)
    e.get_q1_dens_op_with_grad(0)
    e.forward([], [g4])
    with pytest.raises(q.PanicException, match="The number of gradients wrt density matrices is less"):
        e.backward([], [], [g4])
    with pytest.raises(q.PanicException, match="Number of constant gates is more than required."):
        e.backward([np.eye(2, dtype=DT[prec])], [], [g4, g4])  # circuit.rs:426
    with pytest.raises(TypeError):
        e.forward([], [g4.astype(np.complex64 if prec == "f64" else np.complex128)])
    with pytest.raises(q.PanicException, match="Size of the given state does not match"):
        e.set_state_from_vector(np.zeros(4, DT[prec]))


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_zero_grads_before_first_density(prec):
    """circuit.rs:327-331: variable gates after the last Diff density get zero gradients."""
    import quantum_differentiable_circuit as q
    c = q.circuit_class(prec)(4)
    c.add_q1_var_gate(0)
    c.get_q1_dens_op_with_grad(0)
    c.add_q1_var_gate(1)
    g = O.haar_unitary(np.random.default_rng(1), 2).astype(DT[prec])
    c.forward([], [g, g])
    grads = c.backward([np.eye(2, dtype=DT[prec])], [], [g, g])
    assert np.abs(grads[1]).max() == 0
    assert np.abs(grads[0]).max() > 0

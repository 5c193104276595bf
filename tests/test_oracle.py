"""The oracle, pinned against the reference's own known-answer tests (CPU only).

* GHZ amplitudes and densities: primitives.cu:961-1033 (ghz_test), quantized_tensor.rs:487-506,
  test_ghz.py:16-60.
* Inverse KAT: primitives.cu:1035-1073 (inv_test's 3x3 matrix, A A^-1 = I at 1e-5).
* Finite-difference gradient identity: test_autodiff.py:121-165 (8th-order FD, rel 1e-9).
* The einsum restatement (quantized_tensor.rs:287-398) agrees with the C restatement of the
  CUDA kernel index rules (oracle/cpu_ref.c ← primitives.cu) in both precisions.
* The committed golden fixtures are reproduced.
"""
from pathlib import Path

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN = Path(__file__).resolve().parent / "golden"


def test_ghz_primitives_kat():
    """primitives.cu:961-1033 at n = 21 (H, CNOT chain, last CNOT as H.CZ.H)."""
    n = 21
    s = np.zeros(1 << n, np.complex128)
    s[0] = 1
    h = np.array([1, 1, 1, -1]) / np.sqrt(2)
    cnot = np.array([1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 1, 0, 0, 1, 0], np.complex128)
    s = O.apply_q1_gate(s, h, 0)
    for i in range(n - 2):
        s = O.apply_q2_gate(s, cnot, i, i + 1)
    s = O.apply_q1_gate(s, h, n - 1)
    s = O.apply_q2_gate_diag(s, np.array([1, 1, 1, -1]), n - 2, n - 1)
    s = O.apply_q1_gate(s, h, n - 1)
    assert abs(s[0] - 1 / np.sqrt(2)) < 1e-5 and abs(s[-1] - 1 / np.sqrt(2)) < 1e-5
    assert np.abs(s[1:-1]).max() < 1e-5
    for i in range(0, n, 5):
        assert np.abs(O.get_q1_density(s, i) - [.5, 0, 0, .5]).max() < 1e-5
    want = np.zeros(16)
    want[0] = want[15] = .5
    for i in range(0, n - 1, 5):
        assert np.abs(O.get_q2_density(s, i, i + 1) - want).max() < 1e-5


def test_ghz_circuit_kat():
    """test_ghz.py:16-60 through the oracle's Circuit (n reduced to 12; the KATs are n-free)."""
    n = 12
    cnot = np.array([1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 1, 0, 0, 1, 0], np.complex128)
    h = np.array([1, 1, 1, -1], np.complex128) / np.sqrt(2)
    c = O.OracleCircuit(n)
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
    alld = c.run([h] + (n - 1) * [cnot], [])
    diff = c.forward([h] + (n - 1) * [cnot], [])
    assert len(alld) == 2 * n + 2 * (n - 1) and len(diff) == 2 * n - 1
    for a, b in zip(alld[:2 * n - 1], diff):
        assert np.allclose(a, b)
    # test_ghz.py:41: (|+> on pos2 = qubit 0) x (|0> on pos1 = qubit 1), index 2 P2 + P1
    psi = np.tensordot(np.array([1, 1]) / np.sqrt(2), np.array([1., 0.]), axes=0).reshape(4)
    assert np.allclose(np.outer(psi, psi.conj()), alld[0])
    assert np.allclose(alld[n - 1], np.full((2, 2), .5))
    two = np.zeros((4, 4))
    two[0, 0] = two[3, 3] = .5
    for d in alld[3 * n - 1:]:
        assert np.allclose(d, two)


def test_inverse_kat():
    """primitives.cu:1035-1073."""
    a = np.array([1 + 1.1j, 2 + 2j, 3 + 3j, 1.2 + 2.3j, 3.2, 1 + 1.5j, 2.1j, 2 + 4j, 2.11 + 3.44j])
    inv = O.inverse(a).reshape(3, 3)
    assert np.abs(a.reshape(3, 3) @ inv - np.eye(3)).max() < 1e-5


def test_inverse_singular_message():
    with pytest.raises(O.OraclePanic, match=r"U\(1, 1\) is zero\."):
        O.inverse(np.zeros(4))
    with pytest.raises(O.OraclePanic, match=r"U\(2, 2\) is zero\."):
        O.inverse(np.array([1, 2, 2, 4]))


@pytest.mark.parametrize("n,layers", [(5, 2), (6, 3)])
def test_finite_difference_identity(n, layers):
    """test_autodiff.py:121-165 on the oracle: the reverse sweep's gradient g satisfies
    dL = sum Re(g . p) (the JAX cotangent convention)."""
    ins, const, var, pert = O.autodiff_circuit(n, layers, seed=7)
    eta = 1e-6

    def loss(v):
        c = O.OracleCircuit(n)
        for k, pos in ins:
            c.add(k, *pos)
        return O.tsallis_loss_and_cotangents(c.forward(const, v))[0]

    coeff = {-4: 1 / 280, -3: -4 / 105, -2: 1 / 5, -1: -4 / 5, 1: 4 / 5, 2: -1 / 5,
             3: 4 / 105, 4: -1 / 280}
    ds_fd = sum(w * loss([g + k * eta * p for g, p in zip(var, pert)]) for k, w in coeff.items()) / eta
    c = O.OracleCircuit(n)
    for k, pos in ins:
        c.add(k, *pos)
    dens = c.forward(const, var)
    _, cots = O.tsallis_loss_and_cotangents(dens)
    grads = c.backward([x.conj() for x in cots], const, var)  # circuit.py:193 conj
    ds = sum(np.dot(g, p).real for g, p in zip(grads, pert))
    assert abs(ds - ds_fd) / min(abs(ds), abs(ds_fd)) < 1e-8


def test_uncompute_recovers_initial_state():
    ins, var = O.layered_circuit(6, 3, seed=3)
    c = O.OracleCircuit(6)
    for k, pos in ins:
        c.add(k, *pos)
    psi0 = O.random_state(np.random.default_rng(1), 6)
    c.set_state_from_vector(psi0)
    dens = c.forward([], var)
    c.backward([np.eye(2) for _ in dens], [], var)
    assert np.abs(c.state - psi0).max() < 1e-12


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_einsum_matches_kernel_restatement(prec):
    from oracle.cref import CRefOps
    ops = CRefOps(prec)
    tol = 1e-5 if prec == "f32" else 1e-12
    dt = ops.state_dtype
    rng = np.random.default_rng(11)
    n = 9
    s = (rng.random(1 << n) + 1j * rng.random(1 << n)).astype(dt)
    b = (rng.random(1 << n) + 1j * rng.random(1 << n)).astype(dt)
    s128, b128 = s.astype(np.complex128), b.astype(np.complex128)
    for pos in range(n):
        g = (rng.random(4) + 1j * rng.random(4)).astype(dt)
        O.cmp_complex_slices(ops.apply_q1_gate(s.copy(), g, pos), O.apply_q1_gate(s128, g, pos), tol)
        O.cmp_complex_slices(ops.get_q1_density(s, pos), O.get_q1_density(s128, pos), tol)
        O.cmp_complex_slices(ops.get_q1_grad(s, b, pos), O.get_q1_grad(s128, b128, pos), tol)
    for pos2, pos1 in [(0, 1), (1, 0), (0, 8), (8, 0), (3, 5), (5, 3), (7, 8)]:
        g = (rng.random(16) + 1j * rng.random(16)).astype(dt)
        d = (rng.random(4) + 1j * rng.random(4)).astype(dt)
        O.cmp_complex_slices(ops.apply_q2_gate(s.copy(), g, pos2, pos1),
                             O.apply_q2_gate(s128, g, pos2, pos1), tol)
        O.cmp_complex_slices(ops.apply_q2_gate_diag(s.copy(), d, pos2, pos1),
                             O.apply_q2_gate_diag(s128, d, pos2, pos1), tol)
        O.cmp_complex_slices(ops.get_q2_density(s, pos2, pos1), O.get_q2_density(s128, pos2, pos1), tol)
        O.cmp_complex_slices(ops.get_q2_grad(s, b, pos2, pos1), O.get_q2_grad(s128, b128, pos2, pos1), tol)
        O.cmp_complex_slices(ops.get_q2_grad_diag(s, b, pos2, pos1),
                             O.get_q2_grad_diag(s128, b128, pos2, pos1), tol)


def test_cref_circuit_matches_einsum_circuit():
    """The C-backed oracle circuit (the timed CPU baseline) == the einsum oracle circuit."""
    from oracle.cref import CRefOps
    ins, const, var, _ = O.autodiff_circuit(6, 2, seed=9)
    a = O.OracleCircuit(6, np.complex128)
    b = O.OracleCircuit(6, np.complex128, ops=CRefOps("f64"))
    for k, pos in ins:
        a.add(k, *pos)
        b.add(k, *pos)
    da, db = a.forward(const, var), b.forward(const, var)
    for x, y in zip(da, db):
        assert np.abs(x - y).max() < 1e-12
    _, cots = O.tsallis_loss_and_cotangents(da)
    ga = np.concatenate(a.backward([c.conj() for c in cots], const, var))
    gb = np.concatenate(b.backward([c.conj() for c in cots], const, var))
    assert np.abs(ga - gb).max() / np.abs(ga).max() < 1e-12


def test_cmp_complex_slices_metric():
    """test_utils.rs:20-42: relative per element, pairs of exact zeros skipped."""
    O.cmp_complex_slices([0, 1, 2], [0, 1 + 1e-7, 2], 1e-5)
    with pytest.raises(AssertionError):
        O.cmp_complex_slices([1.0], [1.1], 1e-5)


def test_oracle_panics():
    c = O.OracleCircuit(3)
    with pytest.raises(O.OraclePanic, match="The circuit is empty."):
        c.run([], [])
    c.add_q2_var_gate_diag(0, 1)
    with pytest.raises(O.OraclePanic, match="The number of constant gates is less than required."):
        c.run([], [])
    c.forward([], [np.ones(4)])
    with pytest.raises(O.OraclePanic, match="Number of constant gates is more than required."):
        c.backward([], [], [np.ones(4), np.ones(4)])


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_golden_primitives_reproduced(prec):
    z = np.load(GOLDEN / f"primitives_{prec}.npz")
    s = z["state"].astype(np.complex128)
    b = z["bwd"].astype(np.complex128)
    n = int(z["n"])
    for p in range(n):
        assert np.allclose(O.apply_q1_gate(s, z["q1_gates"][p], p), z["q1_out"][p], rtol=1e-12, atol=0)
        assert np.allclose(O.get_q1_grad(s, b, p), z["q1_grad"][p], rtol=1e-12, atol=0)
    for i, (p2, p1) in enumerate(z["pairs"]):
        assert np.allclose(O.apply_q2_gate(s, z["q2_gates"][i], p2, p1), z["q2_out"][i], rtol=1e-12)
        assert np.allclose(O.get_q2_density(s, p2, p1), z["q2_density"][i], rtol=1e-12)


@pytest.mark.parametrize("name", ["circuit_autodiff", "circuit_layered"])
@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_golden_circuits_reproduced(name, prec):
    z = np.load(GOLDEN / f"{name}_{prec}.npz")
    n = int(z["n"])
    split = lambda data, lens: np.split(data, np.cumsum(lens)[:-1]) if len(lens) else []  # noqa
    const, var = split(z["const"], z["const_lens"]), split(z["var"], z["var_lens"])
    o = O.OracleCircuit(n, z["psi0"].dtype)
    for k, a, b in z["instructions"]:
        o.add(int(k), int(a), int(b)) if int(k) in (0, 1, 2, 3, 4, 5, 10, 12) else o.add(int(k), int(a))
    o.set_state_from_vector(z["psi0"])
    fwd = o.forward(const, var)
    want = split(z["forward"], z["forward_lens"])
    assert all(np.allclose(a.reshape(-1), w, rtol=0, atol=1e-6) for a, w in zip(fwd, want))
    cots = [c.reshape(int(np.sqrt(c.size)), -1) for c in split(z["cotangents"], z["cotangent_lens"])]
    grads = np.concatenate(o.backward(cots, const, var))
    assert np.abs(grads - z["grads"]).max() <= 1e-5 * np.abs(z["grads"]).max()


def test_qk_oracle_extends_q1_q2_conventions():
    """apply_qk_gate (dense k-qubit gates, include/qdc/dense.h) has no reference counterpart:
    pin it to the reference's own q1/q2 oracles at k = 1, 2 and to a Kronecker product of
    one-qubit gates (positions[0] = most significant factor) at k = 3."""
    rng = np.random.default_rng(0)
    n = 7
    psi = O.random_state(rng, n)
    for p2, p1 in ((5, 2), (1, 6), (0, 3)):
        g = O.haar_unitary(rng, 4)
        assert np.abs(O.apply_q2_gate(psi, g, p2, p1) - O.apply_qk_gate(psi, g, [p2, p1])).max() < 1e-14
    g1 = O.haar_unitary(rng, 2)
    assert np.abs(O.apply_q1_gate(psi, g1, 3) - O.apply_qk_gate(psi, g1, [3])).max() < 1e-14
    a, b, c = (O.haar_unitary(rng, 2) for _ in range(3))
    u = np.kron(np.kron(a.reshape(2, 2), b.reshape(2, 2)), c.reshape(2, 2))
    want = O.apply_q1_gate(O.apply_q1_gate(O.apply_q1_gate(psi, a, 4), b, 0), c, 6)
    assert np.abs(O.apply_qk_gate(psi, u.reshape(-1), [4, 0, 6]) - want).max() < 1e-14


# --- non-symmetric known answers: every reference KAT uses symmetric matrices (pr.cu:968-978),
# so the row-major U[out, in] convention (quantized_tensor.rs:293), the pos2-MSB quartet order
# (pr.cu:573-606) and the gradient index order (pr.cu:202-292) are pinned here by hand-computed
# values, for both restatements (einsum oracle and the C kernels).
def _kat_ops():
    from oracle.cref import CRefOps
    return [("einsum", O.EinsumOps, np.complex128), ("cref64", CRefOps("f64"), np.complex128),
            ("cref32", CRefOps("f32"), np.complex64)]


@pytest.mark.parametrize("which", [0, 1, 2])
def test_nonsymmetric_kat_conventions(which):
    name, ops, dt = _kat_ops()[which]
    u2 = np.array([1 + 2j, 3 - 1j, -2 + 0.5j, 0.25 + 4j], dt)
    n, pos = 4, 2
    s = np.zeros(1 << n, dt)
    s[0] = 1
    out = ops.apply_q1_gate(s.copy(), u2, pos)
    assert out[0] == u2[0] and out[1 << pos] == u2[2], name  # out[1] = U[2] in[0]
    rho = ops.get_q1_density(out, pos)
    np.testing.assert_allclose(rho, [abs(u2[0]) ** 2, u2[0] * np.conj(u2[2]),
                                     u2[2] * np.conj(u2[0]), abs(u2[2]) ** 2], rtol=1e-6)
    bwd = np.zeros(1 << n, dt)
    bwd[1 << pos] = 1
    g = ops.get_q1_grad(s.copy(), bwd, pos)
    np.testing.assert_array_equal(g, [0, 0, 1, 0])  # G[2p + q], p = bwd's bit, q = fwd's
    u4 = ((np.arange(16) + 1) * (1 + 0.5j)).astype(dt)
    n, pos2, pos1 = 5, 3, 1
    s = np.zeros(1 << n, dt)
    s[0] = 1
    out = ops.apply_q2_gate(s.copy(), u4, pos2, pos1)
    for q2 in (0, 1):
        for q1 in (0, 1):
            assert out[(q2 << pos2) | (q1 << pos1)] == u4[8 * q2 + 4 * q1], (name, q2, q1)
    assert np.count_nonzero(out) == 4

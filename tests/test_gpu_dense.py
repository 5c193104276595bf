"""Dense k-qubit gates (SURVEY.md §8 f rank 4; include/qdc/dense.h, csrc/qdc_qk.hpp): the MFMA
kernel (k = 3..5) and the routed k = 1, 2 paths against the oracle's apply_qk_gate (pinned to
the reference's q1/q2 oracles in tests/test_oracle.py), at every layout class of the targets
(in-chunk qubit 0, lane bits, far bits, unsorted positions), through both kernels; the panics; and at n = 28 the
size-independent round trip U then U^+ (f32 1e-5 / f64 1e-12 norm-relative)."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
DT = {"f32": np.complex64, "f64": np.complex128}
TOL = {"f32": 2e-6, "f64": 1e-13}

POSITIONS = {
    1: [[0], [5], [16]],
    2: [[1, 0], [3, 14], [16, 2]],
    3: [[2, 1, 0], [0, 9, 4], [16, 15, 3], [7, 12, 5]],
    4: [[3, 2, 1, 0], [16, 0, 8, 4], [10, 11, 12, 13], [5, 1, 15, 6]],
    5: [[4, 3, 2, 1, 0], [0, 16, 2, 14, 4], [12, 13, 14, 15, 16], [9, 3, 11, 0, 7]],
}


def tensor(prec, psi):
    import quantum_differentiable_circuit as q
    return q.QuantizedTensor.new_from_host(psi.astype(DT[prec]), precision=prec)


@pytest.mark.parametrize("prec", ["f32", "f64"])
@pytest.mark.parametrize("k", [1, 2, 3, 4, 5])
def test_qk_gate_matches_oracle(prec, k):
    n = 17
    rng = np.random.default_rng(10 + k)
    psi = O.random_state(rng, n)
    for pos in POSITIONS[k]:
        u = O.haar_unitary(rng, 1 << k)
        t = tensor(prec, psi)
        t.apply_qk_gate(u.astype(DT[prec]), pos)
        got = t.get_cpu_state_copy()
        want = O.apply_qk_gate(psi.astype(DT[prec]).astype(np.complex128), u.astype(DT[prec]), pos)
        err = np.abs(got - want).max() / np.abs(want).max()
        assert err < TOL[prec] * 8, (pos, err)


@pytest.mark.parametrize("prec", ["f32", "f64"])
@pytest.mark.parametrize("k", [3, 4, 5])
@pytest.mark.parametrize("lds", ["0", "1"])
def test_qk_gate_both_kernels_every_placement(monkeypatch, prec, k, lds):
    """k_qk (QDC_QK_LDS=0) and the LDS-staged tiles (k_qkl, QDC_QK_LDS=1: every gate with a
    target below qubit 5) at placements that put 0..k targets among the tile's low bits, the
    highest qubit included, and at n = k + 4 (one tile)."""
    monkeypatch.setenv("QDC_QK_LDS", lds)
    rng = np.random.default_rng(40 + k)
    for n, pos in ((17, list(range(k))), (17, list(range(1, k + 1))[::-1]),
                   (17, [4] + list(range(16, 16 - (k - 1), -1))), (17, [0, 5] + list(range(8, 8 + k - 2))),
                   (17, [2, 16] + list(range(10, 10 + k - 2))), (k + 4, list(range(k + 3, 3, -1))),
                   (k + 4, [0] + list(range(k + 3, k + 3 - (k - 1), -1)))):
        psi = O.random_state(rng, n)
        u = O.haar_unitary(rng, 1 << k)
        t = tensor(prec, psi)
        t.apply_qk_gate(u.astype(DT[prec]), pos)
        want = O.apply_qk_gate(psi.astype(DT[prec]).astype(np.complex128), u.astype(DT[prec]), pos)
        err = np.abs(t.get_cpu_state_copy() - want).max() / np.abs(want).max()
        assert err < TOL[prec] * 8, (n, pos, err)


@pytest.mark.parametrize("k", [3, 5])
def test_qk_gate_non_unitary_and_small_states(k):
    """A general (non-unitary) matrix, and states with fewer groups than one MFMA batch."""
    rng = np.random.default_rng(3)
    for n in (k, k + 1, k + 3):
        psi = O.random_state(rng, n)
        u = rng.standard_normal(1 << (2 * k)) + 1j * rng.standard_normal(1 << (2 * k))
        pos = list(rng.permutation(n)[:k])
        t = tensor("f64", psi)
        t.apply_qk_gate(u, pos)
        want = O.apply_qk_gate(psi, u, pos)
        assert np.abs(t.get_cpu_state_copy() - want).max() < 1e-12 * np.abs(want).max()


def test_qk_gate_panics():
    import quantum_differentiable_circuit as q
    t = q.QuantizedTensor.new_standard(6, precision="f32")
    g8 = np.eye(8, dtype=np.complex64).reshape(-1)
    with pytest.raises(q.PanicException, match="positions must be different"):
        t.apply_qk_gate(g8, [1, 2, 1])
    with pytest.raises(q.PanicException, match="out of the bound"):
        t.apply_qk_gate(g8, [1, 2, 6])
    with pytest.raises(q.PanicException, match="Incorrect len"):
        t.apply_qk_gate(np.eye(4, dtype=np.complex64).reshape(-1), [1, 2, 3])
    with pytest.raises(q.PanicException, match="k must be"):
        t.apply_qk_gate(np.eye(64, dtype=np.complex64).reshape(-1), list(range(6)))
    # the C ABI validates too (no Python-side checks on this path)
    lib = q._native.load("f32")
    import ctypes as C
    pos = (C.c_size_t * 3)(0, 0, 1)
    msg = lib.qdc_qkgate(t._p, g8.ctypes.data, pos, 3, 6)
    assert msg is not None and b"different" in msg


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_qk_gate_roundtrip_full_size(prec):
    n = 28 if prec == "f32" else 27
    rng = np.random.default_rng(28)
    import quantum_differentiable_circuit as q
    t = q.QuantizedTensor.new_standard(n, precision=prec)
    # spread the |0> amplitude first, so the round trip is a non-trivial check
    h = (np.array([[1, 1], [1, -1]]) / np.sqrt(2)).astype(DT[prec])
    for p in (0, 7, 20, n - 1):
        t.apply_q1_gate(h.reshape(-1), p)
    before = t.get_cpu_state_copy()
    for k, pos in ((3, [n - 1, 3, 0]), (4, [2, 21, 9, 14]), (5, [0, 1, 2, n - 2, 13])):
        u = O.haar_unitary(rng, 1 << k).reshape(1 << k, 1 << k)
        t.apply_qk_gate(u.reshape(-1).astype(DT[prec]), pos)
        t.apply_qk_gate(u.conj().T.reshape(-1).astype(DT[prec]), pos)
    after = t.get_cpu_state_copy()
    assert np.abs(after - before).max() < (1e-5 if prec == "f32" else 1e-12)

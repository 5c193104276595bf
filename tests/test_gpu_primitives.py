"""GPU parity of the 18 C-ABI primitives against the oracle.

Mirrors the reference's own device-tensor unit tests (src/quantized_tensor.rs:400-609): n = 17,
unnormalised random states and non-unitary random gates with entries uniform in [0, 1) re/im
(quantized_tensor.rs:256-285) — seeded here — and the per-element relative metric of
src/test_utils.rs:20-42.  Tolerances: 1e-5 (f32), 1e-12 (f64) per north_star; the reference's
1e-2 for the inverse round trips (quantized_tensor.rs:424, 462).
"""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

N = 17
TOL = {"f32": 1e-5, "f64": 1e-12}
DT = {"f32": np.complex64, "f64": np.complex128}


@pytest.fixture(params=["f32", "f64"])
def prec(request):
    return request.param


def rnd(rng, size, prec):
    return (rng.random(size) + 1j * rng.random(size)).astype(DT[prec])


def qt(prec):
    import quantum_differentiable_circuit as q
    return q


def test_q1gate(prec):
    q = qt(prec)
    rng = np.random.default_rng(1)
    state = rnd(rng, 1 << N, prec)
    vm = q.QuantizedTensor.new_from_host(state, prec)
    for pos in range(N):
        g = rnd(rng, 4, prec)
        want = O.apply_q1_gate(vm.get_cpu_state_copy().astype(np.complex128), g, pos)
        vm.apply_q1_gate(g, pos)
        O.cmp_complex_slices(vm.get_cpu_state_copy(), want, TOL[prec])


def test_q1gate_inv(prec):
    q = qt(prec)
    rng = np.random.default_rng(2)
    state = rnd(rng, 1 << N, prec)
    vm = q.QuantizedTensor.new_from_host(state, prec)
    for pos in range(N):
        g = rnd(rng, 4, prec)
        vm.apply_q1_gate(g, pos)
        vm.apply_q1_gate_inv(g, pos)
        got = vm.get_cpu_state_copy()
        O.cmp_complex_slices(got, state, 1e-2)
        state = got


def q2_positions(rng, iters=20):
    out = []
    while len(out) < iters:
        p1, p2 = (int(x) for x in rng.integers(0, N, 2))
        if p1 != p2:
            out.append((p2, p1))
    # every layout class: chunk-internal bit 0 as pos1 / pos2, adjacent, far, top
    return out + [(1, 0), (0, 1), (0, N - 1), (N - 1, 0), (N - 1, N - 2), (2, 1), (1, 2)]


def test_q2gate(prec):
    q = qt(prec)
    rng = np.random.default_rng(3)
    vm = q.QuantizedTensor.new_from_host(rnd(rng, 1 << N, prec), prec)
    for pos2, pos1 in q2_positions(rng):
        g = rnd(rng, 16, prec)
        want = O.apply_q2_gate(vm.get_cpu_state_copy().astype(np.complex128), g, pos2, pos1)
        vm.apply_q2_gate(g, pos2, pos1)
        O.cmp_complex_slices(vm.get_cpu_state_copy(), want, TOL[prec])


def test_q2gate_inv(prec):
    q = qt(prec)
    rng = np.random.default_rng(4)
    state = rnd(rng, 1 << N, prec)
    vm = q.QuantizedTensor.new_from_host(state, prec)
    for pos2, pos1 in q2_positions(rng):
        g = rnd(rng, 16, prec)
        vm.apply_q2_gate(g, pos2, pos1)
        vm.apply_q2_gate_inv(g, pos2, pos1)
        got = vm.get_cpu_state_copy()
        O.cmp_complex_slices(got, state, 1e-2)
        state = got


def test_q2gate_diag(prec):
    q = qt(prec)
    rng = np.random.default_rng(5)
    vm = q.QuantizedTensor.new_from_host(rnd(rng, 1 << N, prec), prec)
    for pos2, pos1 in q2_positions(rng):
        g = rnd(rng, 4, prec)
        want = O.apply_q2_gate_diag(vm.get_cpu_state_copy().astype(np.complex128), g, pos2, pos1)
        vm.apply_q2_gate_diag(g, pos2, pos1)
        O.cmp_complex_slices(vm.get_cpu_state_copy(), want, TOL[prec])


def test_ghz(prec):
    """quantized_tensor.rs:487-506 and the CHECK binary's ghz_test (primitives.cu:961-1033)."""
    q = qt(prec)
    from quantum_differentiable_circuit.common_gates import get_cnot, get_hadamard
    n = 21
    h, cnot = get_hadamard(prec), get_cnot(prec)  # common_gates.rs:19-34
    cz = np.array([1, 1, 1, -1], DT[prec])
    vm = q.QuantizedTensor.new_standard(n, prec)
    vm.apply_q1_gate(h, 0)
    for i in range(n - 2):
        vm.apply_q2_gate(cnot, i, i + 1)
    vm.apply_q1_gate(h, n - 1)
    vm.apply_q2_gate_diag(cz, n - 2, n - 1)
    vm.apply_q1_gate(h, n - 1)
    s = vm.get_cpu_state_copy()
    amp = 1 / np.sqrt(2)
    assert abs(s[0] - amp) < 1e-5 and abs(s[-1] - amp) < 1e-5
    assert np.abs(s[1:-1]).max() < 1e-5
    for i in range(n):
        assert np.abs(vm.get_q1_density(i) - np.array([.5, 0, 0, .5])).max() < 1e-5
    want2 = np.zeros(16)
    want2[0] = want2[15] = .5
    for i in range(n - 1):
        assert np.abs(vm.get_q2_density(i, i + 1) - want2).max() < 1e-5


def test_q1density(prec):
    q = qt(prec)
    rng = np.random.default_rng(6)
    state = rnd(rng, 1 << N, prec)
    vm = q.QuantizedTensor.new_from_host(state, prec)
    s = state.astype(np.complex128)
    for i in range(N):
        O.cmp_complex_slices(vm.get_q1_density(i), O.get_q1_density(s, i), TOL[prec])


def test_q2density(prec):
    q = qt(prec)
    rng = np.random.default_rng(7)
    state = rnd(rng, 1 << N, prec)
    vm = q.QuantizedTensor.new_from_host(state, prec)
    s = state.astype(np.complex128)
    for pos2, pos1 in q2_positions(rng):
        O.cmp_complex_slices(vm.get_q2_density(pos2, pos1), O.get_q2_density(s, pos2, pos1),
                             TOL[prec])


def test_grads(prec):
    q = qt(prec)
    rng = np.random.default_rng(8)
    fwd, bwd = rnd(rng, 1 << N, prec), rnd(rng, 1 << N, prec)
    f_vm = q.QuantizedTensor.new_from_host(fwd, prec)
    b_vm = q.QuantizedTensor.new_from_host(bwd, prec)
    f, b = fwd.astype(np.complex128), bwd.astype(np.complex128)
    for pos in range(N):
        O.cmp_complex_slices(q.get_q1_grad(f_vm, b_vm, pos), O.get_q1_grad(f, b, pos), TOL[prec])
    for pos2, pos1 in q2_positions(rng):
        O.cmp_complex_slices(q.get_q2_grad(f_vm, b_vm, pos2, pos1),
                             O.get_q2_grad(f, b, pos2, pos1), TOL[prec])
        O.cmp_complex_slices(q.get_q2_grad_diag(f_vm, b_vm, pos2, pos1),
                             O.get_q2_grad_diag(f, b, pos2, pos1), TOL[prec])


def test_grad_accumulates(prec):
    """The C ABI adds into the caller's buffer (primitives.cu:281-288)."""
    import ctypes as C
    q = qt(prec)
    from quantum_differentiable_circuit._native import ptr
    rng = np.random.default_rng(9)
    f_vm = q.QuantizedTensor.new_from_host(rnd(rng, 1 << 10, prec), prec)
    b_vm = q.QuantizedTensor.new_from_host(rnd(rng, 1 << 10, prec), prec)
    once = q.get_q1_grad(f_vm, b_vm, 3)
    buf = once.copy()
    assert f_vm._lib.q1grad(f_vm._p, b_vm._p, ptr(buf), 3, 10) is None
    O.cmp_complex_slices(buf, 2 * once, TOL[prec] * 10)
    del C


def test_conj_and_double_add_copy(prec):
    q = qt(prec)
    rng = np.random.default_rng(10)
    a, b = rnd(rng, 1 << N, prec), rnd(rng, 1 << N, prec)
    va, vb = q.QuantizedTensor.new_from_host(a, prec), q.QuantizedTensor.new_from_host(b, prec)
    np.testing.assert_array_equal(va.conj_and_double().get_cpu_state_copy(), 2 * a.conj())
    vb.add(va)
    np.testing.assert_array_equal(vb.get_cpu_state_copy(), b + a)
    np.testing.assert_array_equal(va.clone().get_cpu_state_copy(), a)


def test_small_states(prec):
    """Edge sizes: n = 1, 2, 3 touch every chunk-internal layout (f32 packs 2 amplitudes)."""
    q = qt(prec)
    rng = np.random.default_rng(11)
    for n in (1, 2, 3):
        s = rnd(rng, 1 << n, prec)
        vm = q.QuantizedTensor.new_from_host(s, prec)
        for pos in range(n):
            g = rnd(rng, 4, prec)
            want = O.apply_q1_gate(vm.get_cpu_state_copy().astype(np.complex128), g, pos)
            vm.apply_q1_gate(g, pos)
            O.cmp_complex_slices(vm.get_cpu_state_copy(), want, TOL[prec])
            O.cmp_complex_slices(vm.get_q1_density(pos),
                                 O.get_q1_density(vm.get_cpu_state_copy().astype(np.complex128), pos),
                                 TOL[prec])
        for pos2 in range(n):
            for pos1 in range(n):
                if pos1 == pos2:
                    continue
                g = rnd(rng, 16, prec)
                want = O.apply_q2_gate(vm.get_cpu_state_copy().astype(np.complex128), g, pos2, pos1)
                vm.apply_q2_gate(g, pos2, pos1)
                O.cmp_complex_slices(vm.get_cpu_state_copy(), want, TOL[prec])


def test_singular_inverse_message(prec):
    q = qt(prec)
    vm = q.QuantizedTensor.new_standard(4, prec)
    with pytest.raises(q.PanicException, match=r"U\(\d, \d\) is zero\."):
        vm.apply_q1_gate_inv(np.zeros(4, DT[prec]), 0)

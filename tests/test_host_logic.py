"""Host-side wiring without a GPU: the qdc AutoGradCircuit VJP chain (src/qdc/circuit.py:
160-202) driven over the oracle's Circuit in place of the HIP one.  Checks the argument
swap (var, const) -> (const, var), the conjugation of the density cotangents before
Circuit.backward (circuit.py:193) and the (grads, None) return."""
import numpy as np
import pytest

from oracle import oracle as O


class OracleBackedCircuit(O.OracleCircuit):
    def __init__(self, n):
        super().__init__(n, np.complex128)
        self.backward_args = None

    @property
    def dtype(self):
        return np.dtype(np.complex128)

    @dtype.setter
    def dtype(self, v):
        pass

    def backward(self, grads, const, var):
        self.backward_args = [g.copy() for g in grads]
        return super().backward(grads, const, var)


@pytest.fixture
def autograd(monkeypatch):
    import qdc.circuit as qc
    monkeypatch.setattr(qc, "circuit_class", lambda precision=None: OracleBackedCircuit)
    return qc.AutoGradCircuit


def test_vjp_wiring_matches_finite_differences(autograd):
    n = 5
    ins, const, var, pert = O.autodiff_circuit(n, 2, seed=3)
    c = autograd(n)
    for k, pos in ins:
        c.circuit.add(k, *pos)
    simple_run, autodiff_run = c.build()
    dens, pullback = autodiff_run.vjp(var, const)
    loss, cots = O.tsallis_loss_and_cotangents(dens)
    grads, none = pullback(cots)
    assert none is None
    # circuit.py:193: cotangents are conjugated before Circuit.backward
    for sent, cot in zip(c.circuit.backward_args, cots):
        assert np.array_equal(sent, cot.conj())
    eta = 1e-6
    lp = O.tsallis_loss_and_cotangents(autodiff_run([g + eta * p for g, p in zip(var, pert)], const))[0]
    lm = O.tsallis_loss_and_cotangents(autodiff_run([g - eta * p for g, p in zip(var, pert)], const))[0]
    fd = (lp - lm) / (2 * eta)
    ds = sum(np.dot(g, p).real for g, p in zip(grads, pert))
    assert abs(ds - fd) / abs(fd) < 1e-6
    # simple_run returns every density, autodiff_run only the Diff ones
    assert len(simple_run(var, const)) > len(dens)


def test_state_vector_input(autograd):
    c = autograd(3)
    c.add_q1_var_gate(0)
    c.get_q1_dens_op_with_grad(0)
    v = np.zeros(8, np.complex128)
    v[1] = 1
    c.set_state_from_vector(v)
    _, run = c.build()
    (rho,) = run([np.eye(2, dtype=np.complex128).reshape(-1)], [])
    assert np.allclose(rho, [[0, 0], [0, 1]])


@pytest.mark.parametrize("prec,dt,rt", [("f32", np.complex64, np.float32), ("f64", np.complex128, np.float64)])
def test_common_gates(prec, dt, rt):
    """get_hadamard / get_cnot (src/common_gates.rs:19-34) in the build's dtype: row-major,
    1/sqrt(2) formed in the build's float type, CNOT controlled by pos2 (the local MSB)."""
    import quantum_differentiable_circuit as q
    h, cx = q.get_hadamard(prec), q.get_cnot(prec)
    assert h.dtype == dt and cx.dtype == dt and h.shape == (4,) and cx.shape == (16,)
    s = rt(1) / np.sqrt(rt(2))
    assert np.array_equal(h, np.array([s, s, s, -s], dt))
    u = cx.reshape(4, 4)
    assert np.array_equal(u @ u, np.eye(4)) and np.array_equal(u[2:, 2:], [[0, 1], [1, 0]])
    hh = h.astype(np.complex128).reshape(2, 2)
    assert np.abs(hh @ hh - np.eye(2)).max() < (1e-6 if prec == "f32" else 1e-15)
    # the GHZ known answer of the reference (primitives.cu:961-1033) through the oracle
    from oracle import oracle as O
    n = 6
    st = np.zeros(1 << n, np.complex128)
    st[0] = 1
    st = O.apply_q1_gate(st, h.astype(np.complex128), 0)
    for i in range(n - 1):
        st = O.apply_q2_gate(st, cx.astype(np.complex128), i, i + 1)
    assert abs(st[0] - s) < 1e-6 and abs(st[-1] - s) < 1e-6 and np.abs(st[1:-1]).max() == 0


def test_rccl_id_bootstrap_ignores_a_dead_launch(tmp_path):
    """distributed.exchange_id: an id file left by an earlier launch whose rank 0 died is never
    taken (same name, start time within the skew); rank 0 of this launch replaces it."""
    import os
    import struct
    import subprocess
    import sys
    from quantum_differentiable_circuit import distributed as D
    path = tmp_path / "id"
    dead = subprocess.Popen([sys.executable, "-c", "pass"])
    dead.wait()
    now = D.process_start_time()
    host = os.uname().nodename.encode()
    ns = D.pid_namespace()
    path.write_bytes(b"s" * 128 + struct.pack(D._FMT, now, dead.pid, ns, host))
    with pytest.raises(TimeoutError):
        D.exchange_id(1, path, None, timeout=0.3, start=now)
    # a live rank 0 on another host (a shared id path) is taken on its start time alone
    path.write_bytes(b"o" * 128 + struct.pack(D._FMT, now, dead.pid, ns, b"elsewhere"))
    assert D.exchange_id(1, path, None, timeout=1, start=now) == b"o" * 128
    # the same host name but another PID namespace (containers sharing a UTS namespace and
    # /tmp): the pid means nothing here, the start time alone decides
    path.write_bytes(b"p" * 128 + struct.pack(D._FMT, now, dead.pid, ns + 1, host))
    assert D.exchange_id(1, path, None, timeout=1, start=now) == b"p" * 128
    # an unknown namespace (0: /proc/self/ns/pid not readable) on the same host: the old rule,
    # rank 0's pid must be alive
    path.write_bytes(b"z" * 128 + struct.pack(D._FMT, now, dead.pid, 0, host))
    with pytest.raises(TimeoutError):
        D.exchange_id(1, path, None, timeout=0.3, start=now)
    assert D.exchange_id(0, path, lambda: b"n" * 128, start=now) == b"n" * 128
    assert D.exchange_id(1, path, None, timeout=1, start=now) == b"n" * 128
    # an id of a launch that started long before this rank: rejected
    path.write_bytes(b"x" * 128 + struct.pack(D._FMT, now - 1000, os.getpid(), ns, host))
    with pytest.raises(TimeoutError):
        D.exchange_id(1, path, None, timeout=0.3, start=now)

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

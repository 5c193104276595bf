"""The reference's own call sequence through the 18-function C ABI.

A Rust host that links libqdc_{f32,f64}.so per INTEGRATION.md §1 runs circuit.rs:164-429 over
QuantizedTensor: per gate one q1gate / q2gate / q2gate_diag; in the reverse sweep per gate the
uncompute (conj-transpose or true inverse), the gradient reduction with its host sync, the
transposed pull-back, and per density cotangent conj_and_double into a new state + transposed
apply + add.  quantum_differentiable_circuit.abi_circuit.AbiCircuit replays exactly that
sequence; here it runs the test_autodiff.py circuit (all 14 instruction kinds, non-unitary
gates included) in both precisions against the complex128 oracle, within 4x the measured floor
of the same algorithm (tests/floors.py), and against the fused circuit runtime."""
import numpy as np
import pytest

import floors as F
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_abi_replay_autodiff_circuit(prec):
    import quantum_differentiable_circuit as q
    from quantum_differentiable_circuit.abi_circuit import AbiCircuit
    n = 11
    ins, const, var, _ = O.autodiff_circuit(n, 2, seed=17)
    psi0 = O.random_state(np.random.default_rng(2), n)
    fl = F.Floor(prec, n, ins, const, var, psi0=psi0, cots=F.tsallis_cots)
    a = AbiCircuit(n, prec)
    for kind, pos in ins:
        a.add(kind, *pos)
    a.set_state_from_vector(fl.psi0)
    what = f"abi replay {prec} "
    fl.check("run", a.run(fl.const, fl.var), what)
    d = a.forward(fl.const, fl.var)
    fl.check("forward", d, what)
    fl.check("state", a.state.get_cpu_state_copy(), what)
    g = a.backward(fl.cots, fl.const, fl.var)
    fl.check("grads", g, what)
    fl.check("uncomputed", a.state.get_cpu_state_copy(), what)
    fl.check("bwd", a.bwd.get_cpu_state_copy(), what)
    # the fused runtime on the same call sequence
    c = q.circuit_class(prec)(n)
    for kind, pos in ins:
        c._push(kind, *pos)
    c.set_state_from_vector(fl.psi0)
    dc = c.forward(fl.const, fl.var)
    gc_ = c.backward(fl.cots, fl.const, fl.var)
    F.check_pair(prec, dc, d, fl.floor["forward"], f"runtime vs abi replay {prec} forward")
    F.check_pair(prec, gc_, g, fl.floor["grads"], f"runtime vs abi replay {prec} grads")


def test_abi_replay_panics():
    from quantum_differentiable_circuit import PanicException
    from quantum_differentiable_circuit.abi_circuit import AbiCircuit
    a = AbiCircuit(4, "f32")
    with pytest.raises(PanicException, match="The circuit is empty."):
        a.forward([], [])
    a.add(8, 1)
    with pytest.raises(PanicException, match="The number of variable gates is less than required."):
        a.forward([], [])
    u = np.eye(2, dtype=np.complex64).reshape(-1)
    with pytest.raises(PanicException, match="Number of constant gates is more than required."):
        a.forward([u], [u])

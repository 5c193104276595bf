"""The runtime's program trace (qdc_trace_program, host only): every matrix a forward call then a
backward call apply to the forward state, from the runtime's own dry run — the plan, remaps,
permuting passes, fusion into stages and the mirrored reverse sweep — mapped to logical qubits.

Replayed in complex128 on the f64 build's trace, the forward must give the oracle's final state
(src/circuit.rs:164-262) and the backward must undo it (circuit.rs:266-429 uncomputes with U^-1
per gate), on 1, 2 and 8 shards.  This pins the input of the host drift emulator
(tools/drift_trace.py) to what the GPU kernels are given."""
import numpy as np
import pytest

from oracle import oracle as O
from quantum_differentiable_circuit import workloads as W


def _apply(psi, u, qs, n):
    k = len(qs)
    t = psi.reshape((2,) * n)
    ax = [n - 1 - p for p in qs]
    t = np.moveaxis(t, ax, list(range(k))).reshape(1 << k, -1)
    t = u @ t
    return np.moveaxis(t.reshape((2,) * n), list(range(k)), ax).reshape(-1)


def _replay(tr, n, psi, direction):
    for op in tr[tr["dir"] == direction]:
        R = int(op["R"])
        u = np.asarray(op["m"][:R * R], np.complex128).reshape(R, R)
        psi = _apply(psi, u, [int(op["q2"])] if R == 2 else [int(op["q2"]), int(op["q1"])], n)
    return psi


@pytest.mark.parametrize("world", [1, 2, 8])
@pytest.mark.parametrize("circuit", ["deep", "every_kind"])
def test_trace_replays_forward_and_uncompute(world, circuit):
    import quantum_differentiable_circuit as q
    n = 11
    if circuit == "deep":
        ins, var = W.deep_random_circuit(n, 600, seed=4)
        const = []
    else:
        ins, const, var = O.random_circuit(n, 300, seed=9, density_every=50)
    instr = [(k, *p) for k, p in ins]
    cg = [np.ascontiguousarray(g, dtype=np.complex128) for g in const]
    vg = [np.ascontiguousarray(g, dtype=np.complex128) for g in var]
    o = O.OracleCircuit(n, np.complex128)
    for kind, pos in ins:
        o.add(kind, *pos)
    dens = o.forward(cg, vg)
    cots = [np.ascontiguousarray(np.eye(d.shape[0]), dtype=np.complex128) for d in dens]
    tr = q.trace_program(n, instr, cg, vg, cots, world=world, precision="f64")
    fw, bw = tr[tr["dir"] == 0], tr[tr["dir"] == 1]
    assert len(fw) > 0 and len(bw) == len(fw)
    psi0 = np.zeros(1 << n, np.complex128)
    psi0[0] = 1
    psi = _replay(tr, n, psi0, 0)
    assert np.abs(psi - o.state).max() < 1e-12
    back = _replay(tr, n, psi, 1)
    assert np.abs(back - psi0).max() < 1e-10
    # the mirrored sweep: every reverse stage of unitary gates is the adjoint of the forward's
    # recorded matrix (non-unitary stages keep their exact inverse)
    fused = bw[bw["single"] == 0]
    if circuit == "deep":
        assert fused["mirrored"].all()
    elif len(fused):  # (8 shards of 11 qubits leave 8 local ones: no fused tile, single gates)
        assert fused["mirrored"].sum() > 0

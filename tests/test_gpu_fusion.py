"""GPU parity of the fused multi-gate passes.

The runtime groups consecutive gates whose qubits fit one LDS tile into one HBM pass
(`k_fused`, csrc/qdc_kernels.hpp).  Fusion changes the order of floating-point work only
inside a gate (never across gates), so fused and unfused runs must agree with each other and
with the oracle's restatement of src/circuit.rs:164-429 on random circuits over every gate
kind, on arbitrary qubit pairs (row bits of the tile), with densities between the groups.
Tolerances are norm-relative, f32 scaled by depth as in test_gpu_circuit.py."""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
DT = {"f32": np.complex64, "f64": np.complex128}
TOL = {"f32": 3e-4, "f64": 1e-10}


def normrel(a, b):
    a = np.concatenate([np.asarray(x).reshape(-1) for x in a])
    b = np.concatenate([np.asarray(x).reshape(-1) for x in b])
    return np.abs(a - b).max() / np.abs(b).max()


def build(prec, n, ins, fuse, **kw):
    import quantum_differentiable_circuit as q
    old = os.environ.get("QDC_FUSE")
    os.environ["QDC_FUSE"] = str(fuse)
    try:
        c = q.circuit_class(prec)(n, **kw)
    finally:
        if old is None:
            del os.environ["QDC_FUSE"]
        else:
            os.environ["QDC_FUSE"] = old
    for kind, pos in ins:
        c._push(kind, *pos)
    return c


def oracle_pass(n, ins, cg, vg, psi0, dt):
    o = O.OracleCircuit(n, dt)
    for kind, pos in ins:
        o.add(kind, *pos)
    o.set_state_from_vector(psi0)
    dens = o.forward(cg, vg)
    _, cots = O.tsallis_loss_and_cotangents([d.astype(np.complex128) for d in dens])
    cots = [np.ascontiguousarray(x.conj(), dtype=dt) for x in cots]
    grads = o.backward(cots, cg, vg)
    return dens, cots, grads, o.state


@pytest.mark.parametrize("prec", ["f32", "f64"])
@pytest.mark.parametrize("n", [12, 17])
def test_fused_equals_unfused_and_oracle(prec, n):
    dt = DT[prec]
    ins, const, var = O.random_circuit(n, 160, seed=100 + n, density_every=40)
    cg = [g.astype(dt) for g in const]
    vg = [g.astype(dt) for g in var]
    psi0 = O.random_state(np.random.default_rng(n), n).astype(dt)
    dens, cots, grads, final = oracle_pass(n, ins, cg, vg, psi0, dt)
    for fuse in (0, 1):
        c = build(prec, n, ins, fuse)
        c.set_state_from_vector(psi0)
        c.profile(True)
        got = c.forward(cg, vg)
        assert normrel(got, dens) < TOL[prec]
        g = c.backward(cots, cg, vg)
        assert normrel(g, grads) < TOL[prec] * 10
        assert normrel([c.get_state(0)], [final]) < TOL[prec] * 10
        stats = c.profile_collect()
        fused = [k for k in stats if k.startswith("fused")]
        if fuse:
            assert "fused_apply" in stats and "fused_reverse" in stats, sorted(stats)
        else:
            assert not fused, fused


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_fused_brickwork_many_gates_per_pass(prec):
    """C2 brickwork: long fused groups (up to FMAX_OPS) with gradient gates in every group."""
    dt = DT[prec]
    n = 16
    ins, var = O.layered_circuit(n, 4, seed=9)
    vg = [g.astype(dt) for g in var]
    a, b = build(prec, n, ins, 0), build(prec, n, ins, 1)
    b.profile(True)
    da, db = a.forward([], vg), b.forward([], vg)
    assert normrel(db, da) < TOL[prec]
    cots = [np.diag([1.0, -1.0]).astype(dt) for _ in da]
    ga, gb = a.backward(cots, [], vg), b.backward(cots, [], vg)
    assert normrel(gb, ga) < TOL[prec]
    stats = b.profile_collect()
    nfused = stats["fused_reverse"]["launches"]
    ngates = len(var)
    assert nfused * 4 <= ngates, (nfused, ngates)  # >= 4 gates per reverse pass on average


@pytest.mark.parametrize("shards", [2, 8])
def test_fused_with_local_shards(shards):
    """Fusion over the sharded layout (remaps split the groups)."""
    n = 14
    dt = np.complex128
    ins, const, var = O.random_circuit(n, 120, seed=7, density_every=30)
    psi0 = O.random_state(np.random.default_rng(1), n).astype(dt)
    dens, cots, grads, final = oracle_pass(n, ins, const, var, psi0, dt)
    c = build("f64", n, ins, 1, local_shards=shards)
    c.set_state_from_vector(psi0)
    assert normrel(c.forward(const, var), dens) < 1e-10
    assert normrel(c.backward(cots, const, var), grads) < 1e-9
    assert normrel([c.get_state(0)], [final]) < 1e-9

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


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_fused_densities_and_injections_order_rules(prec):
    """Densities / cotangent injections inside fused passes: dense interleaving with
    non-unitary and variable gates on other qubits (the ordering rules), plain densities in
    run mode, and every density batched (no standalone density / injection launches when all
    of them fit tiles)."""
    dt = DT[prec]
    n = 14
    ins, const, var = O.random_circuit(n, 120, seed=321, density_every=3)
    # plain densities too (run mode reports them)
    ins = ins[:20] + [(O.Q1_DENSITY, (3,)), (O.Q2_DENSITY, (9, 2))] + ins[20:]
    cg = [g.astype(dt) for g in const]
    vg = [g.astype(dt) for g in var]
    psi0 = O.random_state(np.random.default_rng(5), n).astype(dt)
    o = O.OracleCircuit(n, dt)
    for kind, pos in ins:
        o.add(kind, *pos)
    o.set_state_from_vector(psi0)
    want_run = o.run(cg, vg)
    dens, cots, grads, final = oracle_pass(n, ins, cg, vg, psi0, dt)
    c = build(prec, n, ins, 1)
    c.set_state_from_vector(psi0)
    assert normrel(c.run(cg, vg), want_run) < TOL[prec]
    assert normrel(c.forward(cg, vg), dens) < TOL[prec]
    assert normrel(c.backward(cots, cg, vg), grads) < TOL[prec] * 10
    assert normrel([c.get_state(0)], [final]) < TOL[prec] * 10


def test_bench_circuit_batches_densities_and_injections():
    import quantum_differentiable_circuit as q
    n = 20
    ins, var = O.layered_circuit(n, 2, seed=3)
    vg = [g.astype(np.complex64) for g in var]
    c = build("f32", n, ins, 1)
    c.profile(True)
    d = c.forward([], vg)
    g = c.backward([np.diag([1.0, -1.0]).astype(np.complex64) for _ in d], [], vg)
    stats = c.profile_collect()
    assert not any(k.startswith(("density", "inject")) for k in stats), sorted(stats)
    ref = build("f32", n, ins, 0)
    d0 = ref.forward([], vg)
    g0 = ref.backward([np.diag([1.0, -1.0]).astype(np.complex64) for _ in d0], [], vg)
    assert normrel(d, d0) < 1e-5 and normrel(g, g0) < 1e-5


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_fused_densities_with_nonunitary_matrices_on_unitary_kinds(prec):
    """The reference applies whatever matrix a unitary-kind gate carries (the FD test perturbs
    them) and uncomputes it with U^+: a density may only pass gates unitary to working
    precision, and in the reverse sweep such inexact gates keep their order relative to
    variable gates, so fused densities and gradients still match the oracle."""
    dt = DT[prec]
    n = 14
    ins, const, var = O.random_circuit(n, 100, seed=77, density_every=2)
    rng = np.random.default_rng(8)
    var = [g + 1e-3 * (rng.standard_normal(g.shape) + 1j * rng.standard_normal(g.shape))
           for g in var]
    cg = [g.astype(dt) for g in const]
    vg = [np.ascontiguousarray(g, dtype=dt) for g in var]
    o = O.OracleCircuit(n, dt)
    for kind, pos in ins:
        o.add(kind, *pos)
    want = o.forward(cg, vg)
    c = build(prec, n, ins, 1)
    assert normrel(c.forward(cg, vg), want) < TOL[prec] / 10
    # reverse sweep: inexact gates keep their order relative to variable gates
    _, cots = O.tsallis_loss_and_cotangents([d.astype(np.complex128) for d in want])
    cots = [np.ascontiguousarray(x.conj(), dtype=dt) for x in cots]
    assert normrel(c.backward(cots, cg, vg), o.backward(cots, cg, vg)) < TOL[prec]


def build_env(prec, n, ins, env):
    import quantum_differentiable_circuit as q
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        c = q.circuit_class(prec)(n)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    for kind, pos in ins:
        c._push(kind, *pos)
    return c


@pytest.mark.parametrize("case", ["layered12", "layered16", "random12", "random17"])
def test_register_resident_passes_equal_lds_passes(case):
    """f32 gate passes run register-resident (k_rq, csrc/qdc_rq.hpp: relayouts through LDS,
    stages on VGPRs) by default; QDC_RQ=0 keeps them in LDS tiles (k_fused).  Both must agree
    with each other and with the oracle, forward and reverse sweep."""
    dt = np.complex64
    kind, n = case[:-2], int(case[-2:])
    if kind == "layered":
        ins, var = O.layered_circuit(n, 4, seed=24)
        const = []
        psi0 = None
    else:
        ins, const, var = O.random_circuit(n, 160, seed=200 + n, density_every=0)
        psi0 = O.random_state(np.random.default_rng(n), n).astype(dt)
    cg = [g.astype(dt) for g in const]
    vg = [g.astype(dt) for g in var]
    res = {}
    for rq in (0, 1):
        c = build_env("f32", n, ins, {"QDC_RQ": rq, "QDC_FUSE": 1})
        if psi0 is not None:
            c.set_state_from_vector(psi0)
        d = c.forward(cg, vg)
        cots = [np.diag([1.0, -1.0]).astype(dt) if x.shape == (2, 2)
                else np.diag([1.0, -1.0, -1.0, 1.0]).astype(dt) for x in d]
        res[rq] = (d, c.backward(cots, cg, vg), cots)
    o = O.OracleCircuit(n, dt)
    for k, pos in ins:
        o.add(k, *pos)
    if psi0 is not None:
        o.set_state_from_vector(psi0)
    want_d = o.forward(cg, vg)
    want_g = o.backward(res[0][2], cg, vg)
    for rq in (0, 1):
        assert normrel(res[rq][0], want_d) < TOL["f32"], rq
        assert normrel(res[rq][1], want_g) < TOL["f32"] * 10, rq
    assert normrel(res[1][1], res[0][1]) < TOL["f32"]


@pytest.mark.parametrize("n", [13, 18])
def test_permuting_passes_equal_fixed_layout(n):
    """f32 gate-only passes permute their tile's qubits on the way out (QDC_RQ_PERM=1, the
    default; later ops run at rewritten positions).  Densities, gradients and the forward and
    uncomputed states (read back in logical order) equal the fixed-layout run and the oracle."""
    dt = np.complex64
    ins, var = O.layered_circuit(n, 5, seed=n)
    vg = [g.astype(dt) for g in var]
    res = {}
    for perm in (0, 1):
        c = build_env("f32", n, ins, {"QDC_RQ_PERM": perm, "QDC_FUSE": 1})
        d = c.forward([], vg)
        fwd_state = c.get_state(0)
        phys = c.layout()[0]
        g = c.backward([np.diag([1.0, -1.0]).astype(dt) for _ in d], [], vg)
        res[perm] = (d, g, fwd_state, c.get_state(0), list(phys))
    assert res[1][4] != list(range(n))  # the permuting run did leave a permuted layout
    o = O.OracleCircuit(n, dt)
    for k, pos in ins:
        o.add(k, *pos)
    want_d = o.forward([], vg)
    want_state = o.state.copy()
    want_g = o.backward([np.diag([1.0, -1.0]).astype(dt) for _ in want_d], [], vg)
    for perm in (0, 1):
        d, g, fs, us, _ = res[perm]
        assert normrel(d, want_d) < TOL["f32"]
        assert normrel(g, want_g) < TOL["f32"] * 10
        assert normrel([fs], [want_state]) < TOL["f32"]
        assert abs(us[0] - 1) < 1e-4 and np.abs(us[1:]).max() < 1e-4

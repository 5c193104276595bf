"""BASELINE.json configs C4 and C5 (SURVEY.md §8 d) on one MI355X.

C4 — n = 30 f32 brickwall, 40 layers of Haar q2 variable gates on (i, i+1), the state sharded
over 4 GPUs in the metric.  Here the 4 shards share the one GPU (loopback transport: the same
planner, pack kernel and block exchange as RCCL, with device copies), at full size, and must
equal the unsharded run; at n = 12 both equal the oracle.

C5 — n = 33 f32 deep random circuit (50 % q1, 35 % q2, 15 % diagonal; DiffQ1Density on
{0, 16, 31, 32}).  At n = 14 with 1000 gates against the oracle; at the full n = 33 (three
64 GiB states resident on one GPU) a 200-gate prefix: density invariants, determinism of a
repeated forward, and the finite-difference identity dL = sum_k Re(G_k . P_k) along a random
gate-space direction (test_autodiff.py:121-165's check, f32 tolerance)."""
import gc

import numpy as np
import pytest

from oracle import oracle as O
from quantum_differentiable_circuit import workloads as W

pytestmark = pytest.mark.gpu


def build(prec, n, ins, **kw):
    import quantum_differentiable_circuit as q
    c = q.circuit_class(prec)(n, **kw)
    for kind, pos in ins:
        c._push(kind, *pos)
    return c


def flat(xs):
    return np.concatenate([np.asarray(x).reshape(-1) for x in xs])


def normrel(a, b):
    a, b = flat(a), flat(b)
    return np.abs(a - b).max() / np.abs(b).max()


def sz_cots(dens, dt):
    return [np.ascontiguousarray(np.diag([1.0, -1.0]).astype(dt)) for _ in dens]


def fwd_bwd(c, vg, dt):
    d = c.forward([], vg)
    return d, c.backward(sz_cots(d, dt), [], vg)


def test_c4_brickwall_small_vs_oracle():
    n = 12
    ins, var = W.brickwall_circuit(n, 6, seed=30)
    vg = [g.astype(np.complex64) for g in var]
    o = O.OracleCircuit(n, np.complex64)
    for kind, pos in ins:
        o.add(kind, *pos)
    dw = o.forward([], vg)
    gw = o.backward(sz_cots(dw, np.complex64), [], vg)
    for shards in (None, 4):
        d, g = fwd_bwd(build("f32", n, ins, local_shards=shards), vg, np.complex64)
        assert normrel(d, dw) < 1e-4 and normrel(g, gw) < 1e-3, shards


def test_c4_brickwall_full_size_sharded_equals_unsharded():
    n, layers = 30, 40
    ins, var = W.brickwall_circuit(n, layers, seed=30)
    vg = [g.astype(np.complex64) for g in var]
    a = build("f32", n, ins)
    da, ga = fwd_bwd(a, vg, np.complex64)
    del a
    gc.collect()
    b = build("f32", n, ins, local_shards=4)
    db, gb = fwd_bwd(b, vg, np.complex64)
    del b
    gc.collect()
    for d in db:
        assert abs(np.trace(d) - 1) < 1e-4
    assert normrel(db, da) < 1e-4
    assert normrel(gb, ga) < 1e-3


def test_c5_deep_random_small_vs_oracle():
    n = 14
    ins, var = W.deep_random_circuit(n, 1000, seed=33)
    vg = [g.astype(np.complex64) for g in var]
    o = O.OracleCircuit(n, np.complex64)
    for kind, pos in ins:
        o.add(kind, *pos)
    dw = o.forward([], vg)
    gw = o.backward(sz_cots(dw, np.complex64), [], vg)
    d, g = fwd_bwd(build("f32", n, ins), vg, np.complex64)
    assert normrel(d, dw) < 3e-4 and normrel(g, gw) < 3e-3


def test_c5_full_size_prefix_invariants_and_fd_identity():
    n = 33
    full, var = W.deep_random_circuit(n, 200, seed=33)
    vg = [g.astype(np.complex64) for g in var]
    c = build("f32", n, full)
    d1, g = fwd_bwd(c, vg, np.complex64)
    assert len(d1) == 4
    for d in d1:
        assert abs(np.trace(d) - 1) < 1e-4
        assert np.abs(d - d.conj().T).max() < 1e-5
        assert np.linalg.eigvalsh((d + d.conj().T) / 2).min() > -1e-4
    assert all(np.isfinite(x).all() for x in g)

    def loss(gates):
        return sum(np.real(np.trace(x @ np.diag([1.0, -1.0]))) for x in c.forward([], gates))

    assert normrel(c.forward([], vg), d1) < 1e-6  # forward restarts from the initial state
    rng = np.random.default_rng(5)
    p = [(rng.standard_normal(x.shape) + 1j * rng.standard_normal(x.shape)).astype(np.complex64)
         for x in vg]
    eps = 1e-2
    lp = loss([(x + eps * y).astype(np.complex64) for x, y in zip(vg, p)])
    lm = loss([(x - eps * y).astype(np.complex64) for x, y in zip(vg, p)])
    fd = (lp - lm) / (2 * eps)
    an = sum(np.real(np.sum(gk.reshape(-1) * pk.reshape(-1))) for gk, pk in zip(g, p))
    scale = np.linalg.norm(flat(g)) * np.linalg.norm(flat(p))
    assert abs(fd - an) <= 2e-3 * scale, (fd, an, scale)
    del c
    gc.collect()

"""Config C5's real shard geometry at depth (BASELINE configs[4]: deep random circuit, 8 shards).

`test_c5_depth_10k_gates_sharded` (tests/test_gpu_mirror.py) runs C5's depth at n = 14, where 8
shards leave 11 local qubits: one fused tile per shard and generic kernels only.  Here the C5
generator runs at n = 26, so 8 shards keep 23 local qubits — the far-row tile geometry,
permuting-pass relabelling, tiled remap packs and the specialized kernels (>= 22 local qubits)
that C5 at n = 33 over 8 GPUs runs — with mirrored sweeps made mandatory (QDC_MIRROR=2):

- 10 000 gates on 8 local shards and on 2 shard streams, generic kernels, against the unsharded
  run of the same circuit: every output within 2 x RATIO x the floor of the reference's own
  algorithm (tests/floors.py) on the same generator and depth at n = 14 (the proxy: the C
  restatement cannot run 10 000 gates at n = 26 in a test's time).  The 2-norm bounds carry the
  parity claim: a rounding random walk's 2-norm relative error depends on the number of
  roundings, not on n; the max-norm lines are printed and held to the same bound.
- the uncompute error ||psi after backward - psi0|| (the O(1)-memory sweep's drift) of every
  configuration within RATIO x the proxy floor.
- 2 000 gates on 8 local shards with the specialized kernels (compiled ahead of time by
  build(): __graft_entry__.PREBUILT) bit-identical to the generic kernels' run (f32).

Reference: the gate-by-gate forward and reverse sweep of src/circuit.rs:164-392.
"""
import gc

import numpy as np
import pytest

import floors as F
from quantum_differentiable_circuit import workloads as W

pytestmark = pytest.mark.gpu

N = 26
DEEP = 10000
SPEC = 2000  # the program __graft_entry__.precompile() compiles for 8 shards
SEED = 33


def _circuit(n, ins, **kw):
    import quantum_differentiable_circuit as q
    c = q.circuit_class("f32")(n, **kw)
    for kind, pos in ins:
        c._push(kind, *pos)
    return c


def _run(ins, var, **kw):
    """forward densities, forward state, gradients, uncomputed state, backward state."""
    vg = [np.ascontiguousarray(g, dtype=np.complex64) for g in var]
    c = _circuit(N, ins, **kw)
    d = c.forward([], vg)
    s = c.get_state(0)
    cots = F.sigma_z_cots(d, np.complex64)
    g = c.backward(cots, [], vg)
    out = {"forward": np.concatenate([x.reshape(-1) for x in d]), "state": s,
           "grads": np.concatenate([x.reshape(-1) for x in g]), "uncomputed": c.get_state(0),
           "bwd": c.get_state(2), "layout_end": c.layout()[0]}
    del c
    gc.collect()
    return out


def _uncompute_error(u):
    e = u.astype(np.complex128)
    e[0] -= 1.0  # psi0 = |0...0>
    return float(np.linalg.norm(e))


@pytest.fixture(scope="module")
def proxy():
    """Floors of the reference's algorithm on the same generator and depth at n = 14."""
    ins, var = W.deep_random_circuit(14, DEEP, seed=SEED)
    return F.Floor("f32", 14, ins, [], var, run=False)


@pytest.fixture(scope="module")
def unsharded():
    ins, var = W.deep_random_circuit(N, DEEP, seed=SEED)
    mp = pytest.MonkeyPatch()
    mp.setenv("QDC_SPEC", "0")
    mp.setenv("QDC_MIRROR", "2")
    try:
        out = _run(ins, var)
    finally:
        mp.undo()
    return ins, var, out


@pytest.mark.parametrize("kw", [{"local_shards": 8}, {"devices": [0, 0]}], ids=["8shards", "2streams"])
def test_c5_n26_10k_gates_sharded_vs_unsharded(monkeypatch, proxy, unsharded, kw):
    ins, var, ref = unsharded
    monkeypatch.setenv("QDC_SPEC", "0")
    monkeypatch.setenv("QDC_MIRROR", "2")  # a backward that did not mirror its forward is an error
    got = _run(ins, var, **kw)
    assert got["layout_end"] == list(range(N)), "every remap undone"
    what = f"C5 n={N} {DEEP} gates {kw} vs unsharded"
    for key in ("forward", "state", "grads", "uncomputed", "bwd"):
        F.check_pair("f32", got[key], ref[key], proxy.floor[key], f"{what} {key} (max-norm)")
        d2 = F.l2rel(got[key], ref[key])
        b2 = 2 * F.RATIO * proxy.floor_l2[key] + 2 * F.ATOL["f32"]
        print(f"[floor-l2] {what} {key}: diff {d2:.3e}  proxy floor {proxy.floor_l2[key]:.3e}  "
              f"bound {b2:.3e}")
        assert d2 <= b2, f"{what} {key}: 2-norm difference {d2:.3e} > {b2:.3e}"
    fl = proxy.floor_l2["uncomputed"]
    for name, u in (("unsharded", ref["uncomputed"]), (str(kw), got["uncomputed"])):
        e = _uncompute_error(u)
        print(f"[drift] C5 n={N} {DEEP} gates {name}: |psi after backward - psi0| = {e:.3e}  "
              f"proxy floor {fl:.3e}  ratio {e / fl:.2f}")
        assert e <= F.RATIO * fl + F.ATOL["f32"], (name, e, fl)


def test_c5_n26_8shards_specialized_bit_identical(monkeypatch):
    """The specialized passes of C5's 8-shard geometry (23 local qubits) against the generic
    kernels on the same program: bit-identical in f32 (same plan, explicit packed FMAs)."""
    import quantum_differentiable_circuit as q
    ins, var = W.deep_random_circuit(N, SPEC, seed=SEED)
    monkeypatch.setenv("QDC_MIRROR", "2")
    monkeypatch.setenv("QDC_SPEC", "0")
    gen = _run(ins, var, local_shards=8)
    monkeypatch.setenv("QDC_SPEC", "1")
    # every kernel synchronously (not the background compiler of programs with more than
    # QDC_SPEC_MAX distinct kernels): loaded from the prebuilt set, or compiled now if missing
    monkeypatch.setenv("QDC_SPEC_MAX", "100000")
    s0 = q.jit_stats("f32")
    spec = _run(ins, var, local_shards=8)
    s1 = q.jit_stats("f32")
    launched = int(s1["launched"] - s0["launched"])
    compiled = int(s1["compiled"] - s0["compiled"])
    print(f"[jit] C5 n={N} {SPEC} gates 8 shards: {launched} specialized launches, "
          f"{compiled} kernels compiled in the test (0: all prebuilt by build())")
    assert s1["enabled"] and launched > 0, s1
    for key in ("forward", "state", "grads", "uncomputed", "bwd"):
        assert np.array_equal(gen[key], spec[key]), f"specialized {key} differs from generic"
    e = _uncompute_error(spec["uncomputed"])
    print(f"[drift] C5 n={N} {SPEC} gates 8 shards specialized: |psi after backward - psi0| = {e:.3e}")

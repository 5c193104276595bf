"""The interleaved state pair (qdc_circuit.hpp `alloc_pair`): an unsharded circuit keeps its
forward and cotangent states in one allocation, alternating in 64 KiB blocks, and every
gate-shaped kernel addresses chunk c of a state at c + (c & gm).  Only addresses change, never
the order of floating-point work, so a circuit must give bit-identical densities, gradients and
states with the pair interleaved (QDC_STATE_ILV=1, the default) and plain (QDC_STATE_ILV=0),
on the single-gate kernels (QDC_FUSE=0) and the fused passes alike; the readbacks (2-D copies
over the blocks) must return exactly the device's physical order at any offset."""
import os

import numpy as np
import pytest

import floors as F
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def build(prec, n, ins, ilv, fuse=1):
    import quantum_differentiable_circuit as q
    env = {"QDC_STATE_ILV": str(ilv), "QDC_FUSE": str(fuse)}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
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


@pytest.mark.parametrize("prec", ["f32", "f64"])
@pytest.mark.parametrize("fuse", [0, 1])
def test_interleaved_pair_bit_identical(prec, fuse):
    # n = 14: 2^13 f32 chunks (the smallest interleaved size), 2^14 f64 chunks
    n = 14
    ins, const, var = O.random_circuit(n, 140, seed=77 + fuse, density_every=35)
    psi0 = O.random_state(np.random.default_rng(3), n)
    fl = F.Floor(prec, n, ins, const, var, psi0=psi0, cots=F.tsallis_cots, run=False)
    out = {}
    for ilv in (1, 0):
        c = build(prec, n, ins, ilv, fuse)
        c.set_state_from_vector(fl.psi0)
        d = c.forward(fl.const, fl.var)
        fwd = c.get_state(0)
        g = c.backward(fl.cots, fl.const, fl.var)
        out[ilv] = (d, fwd, g, c.get_state(0), c.get_state(2))
        if ilv:
            what = f"interleaved n={n} {prec} fuse={fuse} "
            fl.check("forward", d, what)
            fl.check("grads", g, what)
            fl.check("uncomputed", out[ilv][3], what)
        del c
    for name, a, b in zip(("densities", "forward state", "gradients", "uncomputed", "bwd"),
                          out[1], out[0]):
        if isinstance(a, list):
            assert len(a) == len(b)
            for x, y in zip(a, b):
                assert np.array_equal(x, y), f"{name}: interleaved != plain"
        else:
            assert np.array_equal(a, b), f"{name}: interleaved != plain"


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_interleaved_range_reads(prec):
    """qdc_circuit_get_range pieces at offsets and lengths that start, end and span 64 KiB
    blocks of the pair reassemble the physical state get_shard returns, for fwd and bwd."""
    n = 16
    ins, const, var = O.random_circuit(n, 60, seed=5, density_every=20)
    fl = F.Floor(prec, n, ins, const, var, cots=F.tsallis_cots, run=False)
    c = build(prec, n, ins, 1)
    c.forward(fl.const, fl.var)
    c.backward(fl.cots, fl.const, fl.var)
    blk = 4096 * (2 if prec == "f32" else 1)  # amplitudes per 64 KiB block
    cuts = [0, 1, blk - 1, blk, blk + 7, 3 * blk - 5, 5 * blk, (1 << n) - 3, 1 << n]
    for which in (0, 2):
        full = c.get_shard(which, 0)
        parts = [c.get_range(which, a, b - a) for a, b in zip(cuts, cuts[1:])]
        assert np.array_equal(np.concatenate(parts), full), f"state {which}"
        mid = c.get_range(which, blk // 2, 2 * blk + 3)
        assert np.array_equal(mid, full[blk // 2: blk // 2 + 2 * blk + 3])


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_far_target_tile_plans(prec):
    """QDC_TILE_FAR (qdc_device.hpp plan_gate): single-gate ops with no target at chunk bits
    0..5 run on the tile family with every far target as a row bit (reverse ops by default,
    bit 0), or on the direct rows.  n = 17 puts most positions beyond a tile's contiguous bits
    and q2 pairs with one or two far targets.  Every op class on either family (0: all direct,
    7: all tiled) matches the oracle within the measured floors, and the two runs agree."""
    n = 17
    ins, const, var = O.random_circuit(n, 120, seed=41, density_every=30)
    psi0 = O.random_state(np.random.default_rng(8), n)
    fl = F.Floor(prec, n, ins, const, var, psi0=psi0, cots=F.tsallis_cots, run=False)
    res = {}
    # 7w: every class tiled on the widest tiles (QDC_TILE{1,2}_WIDE=2: 2^12 / 2^11 chunks)
    knobs = {0: {"QDC_TILE_FAR": "0"}, 7: {"QDC_TILE_FAR": "7"},
             "7w": {"QDC_TILE_FAR": "7", "QDC_TILE1_WIDE": "2", "QDC_TILE2_WIDE": "2"}}
    for tf, kv in knobs.items():
        old = {k: os.environ.get(k) for k in kv}
        os.environ.update(kv)
        try:
            c = build(prec, n, ins, 1, fuse=0)
        finally:
            for k, v in old.items():
                if v is None:
                    del os.environ[k]
                else:
                    os.environ[k] = v
        c.set_state_from_vector(fl.psi0)
        d = c.forward(fl.const, fl.var)
        fwd = c.get_state(0)
        g = c.backward(fl.cots, fl.const, fl.var)
        what = f"tile_far={tf} n={n} {prec} "
        fl.check("forward", d, what)
        fl.check("state", fwd, what)
        fl.check("grads", g, what)
        fl.check("uncomputed", c.get_state(0), what)
        res[tf] = g
        del c
    F.check_pair(prec, res[7], res[0], fl.floor["grads"], f"n={n} {prec} tiled vs direct grads")
    F.check_pair(prec, res["7w"], res[0], fl.floor["grads"], f"n={n} {prec} wide tiles vs direct grads")

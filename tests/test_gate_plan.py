"""Single-gate launch geometry on CPU (qdc_gate_plan: the runtime's own plan_gate, host only).

A tile-family launch stages 2^(l+h) chunks per state: l contiguous low chunk bits plus h "row"
bits at the global chunk bits hb0 < hb1, and the gate acts on tile-local amplitude bits t1
(pos1) and t2 (pos2).  With QDC_TILE_FAR every target beyond the contiguous bits becomes a row
bit (csrc/qdc_device.hpp plan_gate).  For every q1 position and a spread of q2 pairs, both
ways and for one- and two-state ops:
  * the tiles (tile_base / tile_chunk of csrc/qdc_kernels.hpp, restated here) cover every
    chunk of the state exactly once;
  * each target's tile-local bit addresses exactly that qubit: flipping local amplitude bit
    t of a tile-local index flips global amplitude bit pos;
  * the tile is 2^9 (two states) / 2^10 chunks, or the whole state when it is smaller.
Direct-family plans (no far tile) are checked for their item count."""
import ctypes as C

import numpy as np
import pytest

import quantum_differentiable_circuit as q
from quantum_differentiable_circuit._native import load

LOWBITS = 6


def gate_plan(prec, n, R, pos2, pos1, two, far):
    lib = load(prec)
    out = (C.c_uint * 10)()
    assert lib.qdc_gate_plan(n, R, pos2, pos1, int(two), int(far), out) == 0
    keys = ("tile", "mode", "l", "h", "hb0", "hb1", "t1", "t2", "lo", "hi")
    d = dict(zip(keys, list(out)))
    d["count"] = d["lo"] | (d["hi"] << 32)
    return d


def insert_zero(x, b):
    low = x & ((1 << b) - 1)
    return ((x - low) << 1) | low


def tile_chunks(p, tile):
    """Global chunk index of every tile-local chunk (tile_base + tile_chunk)."""
    l, h = p["l"], p["h"]
    base = tile << l
    if h > 0:
        base = insert_zero(base, p["hb0"])
    if h > 1:
        base = insert_zero(base, p["hb1"])
    c = np.arange(1 << (l + h), dtype=np.int64)
    g = base + (c & ((1 << l) - 1))
    if h > 0:
        g = g + (((c >> l) & 1) << p["hb0"])
    if h > 1:
        g = g + (((c >> (l + 1)) & 1) << p["hb1"])
    return g


def cases(n):
    q1 = [(p, p) for p in range(n)]
    pairs = {(1, 0), (0, 1), (n - 1, n - 2), (n - 2, n - 1), (n - 1, 0), (3, 9), (9, 3)}
    pairs |= {(a, b) for a in range(7, n, 3) for b in range(8, n, 4) if a != b}
    pairs = {(a, b) for a, b in pairs if a < n and b < n and a != b}
    return [(2, a, b) for a, b in q1] + [(4, a, b) for a, b in sorted(pairs)]


@pytest.mark.parametrize("prec", ["f32", "f64"])
@pytest.mark.parametrize("n", [5, 11, 14, 17])
def test_tile_geometry_covers_state_and_targets(prec, n):
    lv = 1 if prec == "f32" else 0
    nch = 1 << (n - lv)
    for R, pos2, pos1 in cases(n):
        for two in (False, True):
            for far in (False, True):
                p = gate_plan(prec, n, R, pos2, pos1, two, far)
                low = any(lv <= x < lv + LOWBITS for x in {pos2, pos1})
                if not p["tile"]:
                    assert not far and not low
                    lo = min(pos2, pos1)
                    items = nch if (R == 2 and lo < lv) else nch // 2 if (R == 2 or lo < lv) \
                        else nch // 4
                    assert p["count"] == items
                    continue
                assert low or far
                T = 9 if two else 10
                cb = (nch.bit_length() - 1)
                assert p["l"] + p["h"] == min(cb, T)
                assert p["h"] <= 2 and (p["h"] < 2 or p["hb0"] < p["hb1"])
                assert p["count"] == nch >> (p["l"] + p["h"])
                seen = np.zeros(nch, np.int32)
                for tile in range(p["count"]):
                    g = tile_chunks(p, tile)
                    seen[g] += 1
                    # tile-local amplitude bit t of each target maps to global amplitude bit pos
                    amp = (g[:, None] << lv) + np.arange(1 << lv)[None, :]
                    amp = amp.reshape(-1)
                    loc = np.arange(amp.size)
                    for t, pos in ((p["t1"], pos1), (p["t2"], pos2)):
                        assert np.array_equal(amp[loc ^ (1 << t)], amp ^ (1 << pos)), \
                            (prec, n, R, pos2, pos1, two, far, p)
                assert (seen == 1).all(), (prec, n, R, pos2, pos1, two, far, p)


def test_gate_plan_rejects_invalid_arguments():
    lib = load("f32")
    out = (C.c_uint * 10)()
    assert lib.qdc_gate_plan(10, 3, 1, 1, 0, 0, out) == -1   # R
    assert lib.qdc_gate_plan(10, 2, 2, 1, 0, 0, out) == -1   # q1 with two positions
    assert lib.qdc_gate_plan(10, 4, 3, 3, 0, 0, out) == -1   # q2 on one qubit
    assert lib.qdc_gate_plan(10, 2, 10, 10, 0, 0, out) == -1  # position out of range

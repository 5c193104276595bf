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


# ---------------------------------------------------------------------------------------
# LANE family (k_lane, csrc/qdc_kernels.hpp): one chunk per lane, partners across lanes.
# ---------------------------------------------------------------------------------------
def lane_plan(prec, n, R, pos2, pos1, reduces=False, blk=False):
    lib = load(prec)
    out = (C.c_uint * 10)()
    rc = lib.qdc_lane_plan(n, R, pos2, pos1, int(reduces) | (2 if blk else 0), out)
    if rc == 1:
        return None
    assert rc == 0
    keys = ("ampk1", "nlow", "nf", "f0", "f1", "m0", "m1", "lo", "hi", "it")
    d = dict(zip(keys, list(out)))
    d["units"] = d["lo"] | (d["hi"] << 32)
    d["ampk"] = d["ampk1"] - 1
    d["ub"] = 10 if blk else 6
    return d


def lane_chunks(p):
    """lane_chunk(g, unit, lane) for every unit and lane: (units, 2^ub) chunk indices."""
    u = np.arange(p["units"], dtype=np.int64)[:, None]
    lane = np.arange(1 << p["ub"], dtype=np.int64)[None, :]
    x = u << p["nlow"]
    if p["nf"] > 0:
        x = insert_zero(x, p["f0"])
    if p["nf"] > 1:
        x = insert_zero(x, p["f1"])
    x = x | (lane & ((1 << p["nlow"]) - 1))
    if p["nf"] > 0:
        x = x | (((lane >> p["nlow"]) & 1) << p["f0"])
    if p["nf"] > 1:
        x = x | (((lane >> (p["nlow"] + 1)) & 1) << p["f1"])
    return x


def lane_emulate(p, R, M, psi, vec):
    """k_lane's arithmetic restated: every lane holds its chunk, gathers the chunks of lanes
    lane ^ mask(d) and computes its own rows with the coefficients M[rr][rr ^ d]; also the
    density accumulators at their absolute (rr, rr ^ d) slots.  Returns (M psi, rho)."""
    ch = lane_chunks(p)
    amps = psi.reshape(-1, vec)[ch]                     # (units, 2^ub, vec)
    lane = np.arange(1 << p["ub"])
    ampk, m0, m1 = p["ampk"], p["m0"], p["m1"]
    rl = np.zeros(lane.size, np.int64)
    if ampk != 0:
        rl |= ((lane & m0) != 0).astype(np.int64)
    if R == 4 and ampk != 1:
        rl |= ((lane & m1) != 0).astype(np.int64) << 1
    out = np.zeros_like(amps)
    rho = np.zeros((R, R), dtype=psi.dtype)
    for v in range(vec):
        rr = rl | ((v << ampk) if ampk >= 0 else 0)
        y = 0
        for d in range(R):
            lm = (m0 if (d & 1) and ampk != 0 else 0) | (m1 if (d & 2) and ampk != 1 else 0)
            vf = v ^ ((d >> ampk) & 1) if ampk >= 0 else v
            partner = amps[:, lane ^ lm, vf]
            y = y + M[rr, rr ^ d][None, :] * partner
            contrib = (amps[:, :, v] * np.conj(partner)).sum(axis=0)
            np.add.at(rho, (rr, rr ^ d), contrib)
        out[:, :, v] = y
    res = psi.copy().reshape(-1, vec)
    res[ch] = out
    return res.reshape(-1), rho


def gate_reference(R, M, psi, n, pos2, pos1):
    i = np.arange(1 << n)
    if R == 2:
        b = (i >> pos1) & 1
        i0 = i & ~(1 << pos1)
        return M[b, 0] * psi[i0] + M[b, 1] * psi[i0 | (1 << pos1)]
    r = ((i >> pos2) & 1) * 2 + ((i >> pos1) & 1)
    base = i & ~((1 << pos2) | (1 << pos1))
    out = 0
    for qq in range(4):
        j = base | (((qq >> 1) & 1) << pos2) | ((qq & 1) << pos1)
        out = out + M[r, qq] * psi[j]
    return out


def density_reference(R, psi, n, pos2, pos1):
    i = np.arange(1 << n)
    r = ((i >> pos1) & 1) if R == 2 else ((i >> pos2) & 1) * 2 + ((i >> pos1) & 1)
    rho = np.zeros((R, R), dtype=psi.dtype)
    base = i & ~((1 << pos2) | (1 << pos1))
    sel = base == i
    for a in range(R):
        for b in range(R):
            ja = base | (((a >> 1) & 1) << pos2 if R == 4 else 0) | ((a & 1) << pos1)
            jb = base | (((b >> 1) & 1) << pos2 if R == 4 else 0) | ((b & 1) << pos1)
            rho[a, b] = (psi[ja[sel]] * np.conj(psi[jb[sel]])).sum()
    return rho


@pytest.mark.parametrize("prec", ["f32", "f64"])
@pytest.mark.parametrize("n,blk", [(7, False), (9, False), (12, False), (11, True), (14, True)])
def test_lane_geometry_covers_state_and_applies_gate(prec, n, blk):
    lv = 1 if prec == "f32" else 0
    vec = 1 << lv
    ub = 10 if blk else 6
    rng = np.random.default_rng(n)
    psi = rng.standard_normal(1 << n) + 1j * rng.standard_normal(1 << n)
    for R, pos2, pos1 in cases(n):
        p = lane_plan(prec, n, R, pos2, pos1, blk=blk)
        if (1 << n) // vec < (1 << ub):
            assert p is None
            continue
        assert p is not None and p["units"] == (1 << (n - lv)) >> ub
        assert p["nlow"] + p["nf"] == ub and (p["nf"] < 2 or p["f0"] < p["f1"])
        ch = lane_chunks(p)
        seen = np.zeros(1 << (n - lv), np.int32)
        np.add.at(seen, ch.reshape(-1), 1)
        assert (seen == 1).all(), (prec, n, R, pos2, pos1, p)
        M = rng.standard_normal((R, R)) + 1j * rng.standard_normal((R, R))
        got, rho = lane_emulate(p, R, M, psi, vec)
        want = gate_reference(R, M, psi, n, pos2, pos1)
        assert np.allclose(got, want, atol=1e-12), (prec, n, R, pos2, pos1, p)
        assert np.allclose(rho, density_reference(R, psi, n, pos2, pos1), atol=1e-9), \
            (prec, n, R, pos2, pos1, p)


def test_lane_plan_reduction_grid_and_invalid_arguments():
    p = lane_plan("f32", 28, 2, 20, 20, reduces=True)
    assert p["units"] == 1 << 21 and p["units"] // (4 * p["it"]) <= 2048
    assert lane_plan("f32", 28, 2, 20, 20)["it"] == 1
    assert lane_plan("f32", 6, 2, 1, 1) is None   # 32 chunks: too small for the family
    lib = load("f32")
    out = (C.c_uint * 10)()
    assert lib.qdc_lane_plan(10, 3, 1, 1, 0, out) == -1
    assert lib.qdc_lane_plan(10, 4, 3, 3, 0, out) == -1

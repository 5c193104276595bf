"""LANE-family single-gate kernels (k_lane: one chunk per lane, partner amplitudes across
lanes; csrc/qdc_kernels.hpp) against the oracle at every target placement of small states:
each q1 position and every ordered q2 pair at n = 7 (one 64-chunk unit in f32), 9, 12 and 14
(the block-wide variant's 1024-chunk units from n = 11 in f32) — targets inside the chunk (f32
qubit 0), at near lane bits and at far lane bits — for gate
application, densities and gradients (primitives.cu:513-646, 689-837, 202-354 via the
primitives ABI).  Tolerances as test_gpu_primitives: 1e-5 (f32), 1e-12 (f64) relative.
The default knob (QDC_LANE=2) runs application and injections on LANE and the other op classes
on the tile / direct families; test_lane_every_op_class repeats the placements with every class
on LANE (QDC_LANE=7), the runtime's reverse kernels included."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

TOL = {"f32": 1e-5, "f64": 1e-12}
DT = {"f32": np.complex64, "f64": np.complex128}


def rnd(rng, size, prec):
    return (rng.random(size) + 1j * rng.random(size)).astype(DT[prec])


def relerr(got, want):
    got = np.asarray(got, dtype=np.complex128).reshape(-1)
    want = np.asarray(want, dtype=np.complex128).reshape(-1)
    return float(np.abs(got - want).max() / max(np.abs(want).max(), 1e-300))


@pytest.mark.parametrize("prec", ["f32", "f64"])
@pytest.mark.parametrize("n", [7, 9, 12, 14])
def test_lane_kernels_every_placement(prec, n):
    bad = _placement_failures(prec, n)
    assert not bad, f"{len(bad)} failing cells: " + "; ".join(bad[:40])


def _placement_failures(prec, n):
    """Every q1 position and ordered q2 pair through the primitives ABI: application, densities
    and gradients against the oracle; the failing cells."""
    import quantum_differentiable_circuit as q
    rng = np.random.default_rng(100 + n)
    st = rnd(rng, 1 << n, prec)
    bw = rnd(rng, 1 << n, prec)
    s64, b64 = st.astype(np.complex128), bw.astype(np.complex128)
    fwd = q.QuantizedTensor.new_from_host(st, prec)
    bwd = q.QuantizedTensor.new_from_host(bw, prec)
    bad = []
    for pos in range(n):
        g = rnd(rng, 4, prec)
        vm = q.QuantizedTensor.new_from_host(st, prec)
        vm.apply_q1_gate(g, pos)
        checks = {
            "apply": (vm.get_cpu_state_copy(), O.apply_q1_gate(s64, g.astype(np.complex128), pos)),
            "density": (fwd.get_q1_density(pos), O.get_q1_density(s64, pos)),
            "grad": (q.get_q1_grad(fwd, bwd, pos), O.get_q1_grad(s64, b64, pos)),
        }
        for k, (got, want) in checks.items():
            e = relerr(got, want)
            if not e <= TOL[prec]:
                bad.append(f"q1 {k} pos={pos} err={e:.2e}")
    for pos2 in range(n):
        for pos1 in range(n):
            if pos2 == pos1:
                continue
            g = rnd(rng, 16, prec)
            vm = q.QuantizedTensor.new_from_host(st, prec)
            vm.apply_q2_gate(g, pos2, pos1)
            checks = {
                "apply": (vm.get_cpu_state_copy(),
                          O.apply_q2_gate(s64, g.astype(np.complex128), pos2, pos1)),
                "density": (fwd.get_q2_density(pos2, pos1), O.get_q2_density(s64, pos2, pos1)),
                "grad": (q.get_q2_grad(fwd, bwd, pos2, pos1), O.get_q2_grad(s64, b64, pos2, pos1)),
            }
            for k, (got, want) in checks.items():
                e = relerr(got, want)
                if not e <= TOL[prec]:
                    bad.append(f"q2 {k} ({pos2},{pos1}) err={e:.2e}")
    return bad


def _reverse_failures(prec, n, diag_only=False):
    """The runtime's single-gate reverse kernels (uncompute + gradient + pull-back, fusion off)
    at every q1 position and ordered q2 pair (dense and diagonal; diag_only: a q1 layer and the
    diagonal pairs): gradients and the uncomputed state against the oracle's circuit
    (src/circuit.rs:266-429)."""
    import quantum_differentiable_circuit as q
    rng = np.random.default_rng(7 + n)
    ins, var = [], []
    for pos in range(n):
        ins.append((O.VAR_Q1, (pos,)))
        var.append(O.haar_unitary(rng, 2))
    for pos2 in range(n):
        for pos1 in range(n):
            if pos2 != pos1:
                if not diag_only:
                    ins.append((O.VAR_Q2, (pos2, pos1)))
                    var.append(O.haar_unitary(rng, 4))
                ins.append((O.VAR_Q2_DIAG, (pos2, pos1)))
                var.append(np.exp(1j * rng.standard_normal(4)))
    ins += [(O.DIFF_Q1_DENSITY, (p,)) for p in range(n)]
    vg = [np.ascontiguousarray(g, dtype=DT[prec]) for g in var]
    c = q.circuit_class(prec)(n)
    o = O.OracleCircuit(n)
    for kind, pos in ins:
        c._push(kind, *pos)
        o.add(kind, *pos)
    d = c.forward([], vg)
    od = o.forward([], [g.astype(np.complex128) for g in vg])
    cots = [np.ascontiguousarray(np.diag([1.0, -1.0]), dtype=DT[prec]) for _ in d]
    g = np.concatenate([x.reshape(-1) for x in c.backward(cots, [], vg)])
    og = np.concatenate([np.asarray(x).reshape(-1) for x in
                         o.backward([x.astype(np.complex128) for x in cots], [],
                                    [g.astype(np.complex128) for g in vg])])
    bad = []
    # (a circuit of n + 2 n (n - 1) gates: the f32 rounding grows with its depth)
    tol = TOL[prec] * (20 if prec == "f32" else 1)
    for k, got, want in (("densities", np.concatenate([x.reshape(-1) for x in d]),
                          np.concatenate([np.asarray(x).reshape(-1) for x in od])),
                         ("grads", g, og), ("uncomputed", c.get_state(0), o.state)):
        e = relerr(got, want)
        if not e <= tol:
            bad.append(f"reverse {k} err={e:.2e}")
    return bad


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_lane_every_op_class(prec):
    """QDC_LANE=7: every single-gate op class on the LANE family — application and injections
    (the default), the reverse with its gradient (bit 0) and densities and gradients (bit 2) —
    against the oracle at every placement (n = 9: in-chunk, near and far lane bits; n = 12: the
    block-wide variant), through the primitives ABI and the runtime with fusion off.  In a child
    process: the knob is read when a device context is created (qdc_device.hpp)."""
    import json
    import os
    import subprocess
    import sys
    from pathlib import Path
    here = Path(__file__).resolve().parent
    code = (f"import sys, json; sys.path[:0] = [{str(here)!r}, {str(here.parent)!r}, "
            f"{str(here.parent / 'differentiable-quantum-circuit-cuda_amd')!r}]\n"
            "import test_gpu_lane as t\n"
            f"bad = []\n"
            f"for n in (9, 12):\n"
            f"    bad += t._placement_failures({prec!r}, n) + t._reverse_failures({prec!r}, n)\n"
            "print(json.dumps(bad))\n")
    env = dict(os.environ, QDC_LANE="7", QDC_FUSE="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    bad = json.loads(r.stdout.strip().splitlines()[-1])
    print(f"[lane] QDC_LANE=7 {prec}: {len(bad)} failing cells")
    assert not bad, f"{len(bad)} failing cells: " + "; ".join(bad[:40])


@pytest.mark.parametrize("prec", ["f32", "f64"])
@pytest.mark.parametrize("n", [14, 16])
def test_diag_reverse_every_pair(prec, n, monkeypatch):
    """The diagonal reverse kernel with k fixed per thread (k_diag_q, qdc_kernels.hpp; 16 chunks
    in flight per thread, so a block spans 4096 chunks): at n = 16 the state splits into whole
    blocks per quadrant for every ordered pair, at n = 14 for the pairs with at most one block
    bit in f32 (both in f64; the others run k_diag) — positions at the in-chunk amplitude bit, at
    thread chunk bits (< 8) and at block chunk bits (one or both: quadrant walks) — uncompute,
    gradient and pull-back against the oracle's circuit, fusion off (primitives.cu:649-672 via
    circuit.rs:320-392)."""
    monkeypatch.setenv("QDC_FUSE", "0")
    bad = _reverse_failures(prec, n, diag_only=True)
    assert not bad, "; ".join(bad)


def _large_circuit(n, seed=5):
    """The gate list of _large_reverse and its seeded matrices."""
    rng = np.random.default_rng(seed)
    ins = [(O.VAR_Q1, (p,)) for p in (0, 1, 3, 5, n - 5)]
    ins += [(O.VAR_Q2, pr) for pr in ((0, 1), (1, 2), (3, 5), (5, 2), (n - 1, 4))]
    ins += [(O.VAR_Q2_DIAG, pr) for pr in ((0, 1), (n - 5, n - 1), (2, 9))]
    ins += [(O.DIFF_Q1_DENSITY, (0,)), (O.DIFF_Q1_DENSITY, (n - 1,))]
    var = []
    for k, _ in ins:
        if k == O.VAR_Q1:
            var.append(O.haar_unitary(rng, 2))
        elif k == O.VAR_Q2:
            var.append(O.haar_unitary(rng, 4))
        elif k == O.VAR_Q2_DIAG:
            var.append(np.exp(1j * rng.standard_normal(4)))
    return ins, var


def _large_reverse(prec, n):
    """A short circuit at a size whose reducing tile launches give each block several tiles
    (n = 25 f32: 8192 two-state tiles on 4096 blocks): q1 / q2 / diagonal gates at low
    positions (tiles without row bits: the pipelined path), at far positions (row bits) and a
    far-far diagonal pair; densities at 0 and n - 1.  Returns the densities, gradients and the
    uncomputed state (fusion off: the single-gate reverse kernels)."""
    import quantum_differentiable_circuit as q
    ins, var = _large_circuit(n)
    vg = [np.ascontiguousarray(g, dtype=DT[prec]) for g in var]
    c = q.circuit_class(prec)(n)
    for kind, pos in ins:
        c._push(kind, *pos)
    d = c.forward([], vg)
    cots = [np.ascontiguousarray(np.diag([1.0, -1.0]), dtype=DT[prec]) for _ in d]
    g = c.backward(cots, [], vg)
    return d, g, c.get_state(0)


@pytest.mark.parametrize("prec,n", [("f32", 25), ("f64", 24)])
def test_reverse_pipelined_tiles_large_state(prec, n):
    """Tile-family blocks with several tiles load the next tile during this tile's math
    (QDC_TILE_PF, round 6; only reachable at large states): the single-gate reverse sweep with
    it and without it must agree bit for bit, and both with the oracle's circuit
    (src/circuit.rs:266-429).  Child processes: the knob is read at context creation."""
    import os
    import subprocess
    import sys
    import tempfile
    from pathlib import Path
    here = Path(__file__).resolve().parent
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for pf in ("0", "1"):
            f = os.path.join(td, f"pf{pf}.npz")
            code = (f"import sys; sys.path[:0] = [{str(here)!r}, {str(here.parent)!r}, "
                    f"{str(here.parent / 'differentiable-quantum-circuit-cuda_amd')!r}]\n"
                    "import numpy as np, test_gpu_lane as t\n"
                    f"d, g, st = t._large_reverse({prec!r}, {n})\n"
                    f"np.savez({f!r}, d=np.concatenate([np.asarray(x).reshape(-1) for x in d]), "
                    "g=np.concatenate([np.asarray(x).reshape(-1) for x in g]), st=st)\n")
            env = dict(os.environ, QDC_FUSE="0", QDC_TILE_PF=pf)
            r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True,
                               text=True, timeout=300)
            assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
            with np.load(f) as z:
                out[pf] = {k: z[k] for k in ("d", "g", "st")}
    for k in ("d", "g", "st"):
        assert np.array_equal(out["0"][k], out["1"][k]), f"{k} differs with the pipelined tiles"
    # the oracle on the same circuit (the working-precision matrices, as uploaded)
    ins, var = _large_circuit(n)
    o = O.OracleCircuit(n)
    for kind, pos in ins:
        o.add(kind, *pos)
    vg = [np.asarray(g, dtype=DT[prec]).astype(np.complex128) for g in var]
    od = o.forward([], vg)
    og = o.backward([np.diag([1.0, -1.0]).astype(np.complex128) for _ in od], [], vg)
    tol = TOL[prec] * (20 if prec == "f32" else 1)
    for k, got, want in (("densities", out["1"]["d"], np.concatenate([np.asarray(x).reshape(-1) for x in od])),
                         ("grads", out["1"]["g"], np.concatenate([np.asarray(x).reshape(-1) for x in og])),
                         ("uncomputed", out["1"]["st"], o.state)):
        e = relerr(got, want)
        print(f"[pf-tiles] {prec} n={n} {k} err={e:.2e}")
        assert e <= tol, f"{k} err={e:.2e}"

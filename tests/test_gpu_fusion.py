"""GPU parity of the fused multi-gate passes.

The runtime groups gates whose qubits fit one tile into one HBM pass (`k_fused`, `k_rq`), and
inside a pass multiplies runs of gates on one qubit pair into one register stage (a host-formed
product in double, qdc_stage.hpp); gates on disjoint qubits may run in another order.  So fused
and unfused runs differ in floating-point rounding across gates, not only inside one: both must
stay within 4x the measured floor of the reference's own algorithm on the same circuit
(tests/floors.py) against the complex128 oracle's restatement of src/circuit.rs:164-429, on
random circuits over every gate kind, on arbitrary qubit pairs (row bits of the tile), with
densities between the groups; two HIP runs of one circuit differ by at most 8x the floor."""
import os
from pathlib import Path

import numpy as np
import pytest

import floors as F
from oracle import oracle as O

pytestmark = pytest.mark.gpu
DT = {"f32": np.complex64, "f64": np.complex128}


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


@pytest.mark.parametrize("prec", ["f32", "f64"])
@pytest.mark.parametrize("n", [12, 17])
def test_fused_equals_unfused_and_oracle(prec, n):
    ins, const, var = O.random_circuit(n, 160, seed=100 + n, density_every=40)
    psi0 = O.random_state(np.random.default_rng(n), n)
    fl = F.Floor(prec, n, ins, const, var, psi0=psi0, cots=F.tsallis_cots, run=False)
    for fuse in (0, 1):
        c = build(prec, n, ins, fuse)
        c.set_state_from_vector(fl.psi0)
        c.profile(True)
        what = f"random n={n} {prec} fuse={fuse} "
        fl.check("forward", c.forward(fl.const, fl.var), what)
        fl.check("grads", c.backward(fl.cots, fl.const, fl.var), what)
        fl.check("uncomputed", c.get_state(0), what)
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
    fl = F.Floor(prec, n, ins, [], var, run=False)
    a, b = build(prec, n, ins, 0), build(prec, n, ins, 1)
    b.profile(True)
    da, db = a.forward([], fl.var), b.forward([], fl.var)
    fl.check("forward", db, f"brickwork n={n} {prec} fused ")
    F.check_pair(prec, db, da, fl.floor["forward"], f"brickwork n={n} {prec} fused vs unfused forward")
    ga, gb = a.backward(fl.cots, [], fl.var), b.backward(fl.cots, [], fl.var)
    fl.check("grads", gb, f"brickwork n={n} {prec} fused ")
    F.check_pair(prec, gb, ga, fl.floor["grads"], f"brickwork n={n} {prec} fused vs unfused grads")
    stats = b.profile_collect()
    nfused = stats["fused_reverse"]["launches"]
    ngates = len(var)
    assert nfused * 4 <= ngates, (nfused, ngates)  # >= 4 gates per reverse pass on average

@pytest.mark.parametrize("shards", [2, 8])
def test_fused_with_local_shards(shards):
    """Fusion over the sharded layout (remaps split the groups)."""
    n = 14
    ins, const, var = O.random_circuit(n, 120, seed=7, density_every=30)
    psi0 = O.random_state(np.random.default_rng(1), n)
    fl = F.Floor("f64", n, ins, const, var, psi0=psi0, cots=F.tsallis_cots, run=False)
    c = build("f64", n, ins, 1, local_shards=shards)
    c.set_state_from_vector(fl.psi0)
    what = f"random n={n} f64 {shards} shards "
    fl.check("forward", c.forward(fl.const, fl.var), what)
    fl.check("grads", c.backward(fl.cots, fl.const, fl.var), what)
    fl.check("uncomputed", c.get_state(0), what)

@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_fused_densities_and_injections_order_rules(prec):
    """Densities / cotangent injections inside fused passes: dense interleaving with
    non-unitary and variable gates on other qubits (the ordering rules), plain densities in
    run mode, and every density batched (no standalone density / injection launches when all
    of them fit tiles)."""
    n = 14
    ins, const, var = O.random_circuit(n, 120, seed=321, density_every=3)
    # plain densities too (run mode reports them)
    ins = ins[:20] + [(O.Q1_DENSITY, (3,)), (O.Q2_DENSITY, (9, 2))] + ins[20:]
    psi0 = O.random_state(np.random.default_rng(5), n)
    fl = F.Floor(prec, n, ins, const, var, psi0=psi0, cots=F.tsallis_cots)
    c = build(prec, n, ins, 1)
    c.set_state_from_vector(fl.psi0)
    what = f"order rules n={n} {prec} "
    fl.check("run", c.run(fl.const, fl.var), what)
    fl.check("forward", c.forward(fl.const, fl.var), what)
    fl.check("grads", c.backward(fl.cots, fl.const, fl.var), what)
    fl.check("uncomputed", c.get_state(0), what)

def test_bench_circuit_batches_densities_and_injections():
    n = 20
    ins, var = O.layered_circuit(n, 2, seed=3)
    fl = F.Floor("f32", n, ins, [], var, run=False)
    c = build("f32", n, ins, 1)
    c.profile(True)
    d = c.forward([], fl.var)
    g = c.backward(fl.cots, [], fl.var)
    stats = c.profile_collect()
    # densities in fused passes; the sigma-z cotangents are diagonal, so their injections run
    # as one elementwise pass (QDC_DIAG_INJECT), never as single-gate injections
    assert not any(k.startswith(("density", "inject")) and k != "inject_diag" for k in stats), sorted(stats)
    assert stats["inject_diag"]["launches"] == 1, sorted(stats)
    fl.check("forward", d, f"C2 n={n} f32 ")
    fl.check("grads", g, f"C2 n={n} f32 ")
    ref = build("f32", n, ins, 0)
    d0 = ref.forward([], fl.var)
    g0 = ref.backward(fl.cots, [], fl.var)
    F.check_pair("f32", d, d0, fl.floor["forward"], f"C2 n={n} fused vs unfused forward")
    F.check_pair("f32", g, g0, fl.floor["grads"], f"C2 n={n} fused vs unfused grads")

@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_fused_densities_with_nonunitary_matrices_on_unitary_kinds(prec):
    """The reference applies whatever matrix a unitary-kind gate carries (the FD test perturbs
    them) and uncomputes it with U^+: a density may only pass gates unitary to working
    precision, and in the reverse sweep such inexact gates keep their order relative to
    variable gates, so fused densities and gradients still match the oracle."""
    n = 14
    ins, const, var = O.random_circuit(n, 100, seed=77, density_every=2)
    rng = np.random.default_rng(8)
    var = [g + 1e-3 * (rng.standard_normal(g.shape) + 1j * rng.standard_normal(g.shape))
           for g in var]
    fl = F.Floor(prec, n, ins, const, var, cots=F.tsallis_cots, run=False)
    c = build(prec, n, ins, 1)
    what = f"non-unitary unitary-kind n={n} {prec} "
    fl.check("forward", c.forward(fl.const, fl.var), what)
    # reverse sweep: inexact gates keep their order relative to variable gates
    fl.check("grads", c.backward(fl.cots, fl.const, fl.var), what)

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


# register-resident variants (csrc/qdc_rq.hpp): k_rq (a tile per block of NT threads, QDC_RW=0),
# k_rw (a tile per wave; bit 0 two-state, bit 1 one-state, bit 2 two-state with the next tile
# prefetched into AGPRs), the grid-strided tile order, and block-contiguous tiles in XCD-aware
# block order
RQ_VARIANTS = {
    "lds": {"QDC_RQ": 0},
    "k_rq": {"QDC_RQ": 1, "QDC_RW": 0},
    "k_rw": {"QDC_RQ": 1, "QDC_RW": 1},
    "k_rw_all": {"QDC_RQ": 1, "QDC_RW": 3},
    "k_rw_pf": {"QDC_RQ": 1, "QDC_RW": 5},
    "k_rw_gstride": {"QDC_RQ": 1, "QDC_RW": 1, "QDC_RQ_ORDER": 1},
    "k_rw_xcd": {"QDC_RQ": 1, "QDC_RW": 1, "QDC_RQ_ORDER": 2},
}


@pytest.mark.parametrize("case", ["layered12", "layered16", "random12", "random17"])
def test_register_resident_passes_equal_lds_passes(case):
    """f32 gate passes run register-resident (csrc/qdc_rq.hpp: relayouts through LDS, stages
    on VGPRs) by default; QDC_RQ=0 keeps them in LDS tiles (k_fused).  Every variant of
    RQ_VARIANTS must agree with the oracle and with the LDS passes, forward and reverse sweep."""
    kind, n = case[:-2], int(case[-2:])
    if kind == "layered":
        ins, var = O.layered_circuit(n, 4, seed=24)
        const = []
        psi0 = None
    else:
        ins, const, var = O.random_circuit(n, 160, seed=200 + n, density_every=0)
        psi0 = O.random_state(np.random.default_rng(n), n)
    fl = F.Floor("f32", n, ins, const, var, psi0=psi0, run=False)
    res = {}
    for name, env in RQ_VARIANTS.items():
        c = build_env("f32", n, ins, dict(env, QDC_FUSE=1))
        if psi0 is not None:
            c.set_state_from_vector(fl.psi0)
        d = c.forward(fl.const, fl.var)
        g = c.backward(fl.cots, fl.const, fl.var)
        what = f"{case} {name} "
        fl.check("forward", d, what)
        fl.check("grads", g, what)
        fl.check("uncomputed", c.get_state(0), what)
        res[name] = (d, g)
    for name in RQ_VARIANTS:
        if name != "lds":
            F.check_pair("f32", res[name][1], res["lds"][1], fl.floor["grads"],
                         f"{case} {name} vs lds grads")


@pytest.mark.parametrize("n,perm_low,lcmin",
                         [(13, 0, 0), (18, 0, 0), (18, 6, 0), (18, 8, 0), (18, 5, 4), (18, 6, 5)])
def test_permuting_passes_equal_fixed_layout(n, perm_low, lcmin):
    """f32 gate-only passes permute their tile's qubits on the way out (QDC_RQ_PERM=1, the
    default; later ops run at rewritten positions).  Densities, gradients and the forward and
    uncomputed states (read back in logical order) equal the fixed-layout run and the oracle.
    QDC_RQ_PERM_LOW (low positions a permuting pass fills; 0 = the default LV + 3) 6 and 8 move
    qubits to tile bits >= 4, stored through the dest-mapped layout (qdc_fusion.hpp rq_hbm);
    with QDC_FUSE_LCMIN 4 / 5 (256-B / 512-B tile rows) those bits are contiguous chunk bits."""
    ins, var = O.layered_circuit(n, 5, seed=n)
    fl = F.Floor("f32", n, ins, [], var, run=False)
    res = {}
    for perm in (0, 1):
        env = {"QDC_RQ_PERM": perm, "QDC_FUSE": 1}
        if perm_low:
            env["QDC_RQ_PERM_LOW"] = perm_low
        if lcmin:
            env["QDC_FUSE_LCMIN"] = lcmin
        c = build_env("f32", n, ins, env)
        d = c.forward([], fl.var)
        fwd_state = c.get_state(0)
        phys = c.layout()[0]
        g = c.backward(fl.cots, [], fl.var)
        res[perm] = (d, g, fwd_state, c.get_state(0), list(phys))
    assert res[1][4] != list(range(n))  # the permuting run did leave a permuted layout
    for perm in (0, 1):
        d, g, fs, us, _ = res[perm]
        what = f"layered n={n} perm={perm} perm_low={perm_low} lcmin={lcmin} "
        fl.check("forward", d, what)
        fl.check("grads", g, what)
        fl.check("state", fs, what)
        fl.check("uncomputed", us, what)


@pytest.mark.parametrize("case", ["layered12", "random12", "random15"])
def test_f64_register_resident_passes_equal_lds_passes(case):
    """f64 gate passes run register-resident too (k_rw: one wave per 2^10-amplitude two-state
    tile, four VGPRs per amplitude, HBM layouts with tile bits 0..2 as thread bits since a
    16-B chunk is one amplitude).  QDC_RQ64=0 keeps them on the LDS tiles; both agree with the
    oracle within 4x the f64 floor and with each other."""
    kind, n = case[:-2], int(case[-2:])
    if kind == "layered":
        ins, var = O.layered_circuit(n, 4, seed=25)
        const, psi0 = [], None
    else:
        ins, const, var = O.random_circuit(n, 160, seed=300 + n, density_every=0)
        psi0 = O.random_state(np.random.default_rng(n + 1), n)
    fl = F.Floor("f64", n, ins, const, var, psi0=psi0, run=False)
    res = {}
    for rq64 in (1, 0):
        c = build_env("f64", n, ins, {"QDC_RQ64": rq64, "QDC_FUSE": 1})
        if psi0 is not None:
            c.set_state_from_vector(fl.psi0)
        d = c.forward(fl.const, fl.var)
        g = c.backward(fl.cots, fl.const, fl.var)
        what = f"{case} f64 QDC_RQ64={rq64} "
        fl.check("forward", d, what)
        fl.check("grads", g, what)
        fl.check("uncomputed", c.get_state(0), what)
        res[rq64] = g
    F.check_pair("f64", res[1], res[0], fl.floor["grads"], f"{case} f64 k_rw vs lds grads")


def _with_env(env, make):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return make()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_dynamic_tail_is_deterministic(prec):
    """Reverse passes with a dynamic tail (tiles handed out by atomic counters, so which wave
    runs which tile changes from run to run) give bit-identical densities, gradients and states
    on every call: each granule of dynamic tiles reduces into its own partial, summed in a fixed
    order (qdc_rq.hpp k_rw, k_dsum, k_finalize).  Against static shares only (QDC_DYN=100) the
    results differ by rounding: within the north star's tolerance."""
    import quantum_differentiable_circuit as q
    n = 24 if prec == "f32" else 23  # >= 4 x 2048 tiles, so the tail is on
    ins, var = O.layered_circuit(n, layers=2, seed=5)
    dt = DT[prec]
    vg = [np.ascontiguousarray(g, dtype=dt) for g in var]
    cots = F.sigma_z_cots([np.zeros((2, 2))] * n, dt)

    def once(env):
        c = _with_env(env, lambda: q.circuit_class(prec)(n))
        for kind, pos in ins:
            c._push(kind, *pos)
        d = c.forward([], vg)
        g = c.backward(cots, [], vg)
        d2 = c.forward([], vg)
        g2 = c.backward(cots, [], vg)
        return np.concatenate([x.reshape(-1) for x in d]), np.concatenate(g), \
            np.concatenate([x.reshape(-1) for x in d2]), np.concatenate(g2), c.get_state(2)

    d1, g1, d1b, g1b, b1 = once({"QDC_DYN": "35"})
    assert np.array_equal(d1, d1b) and np.array_equal(g1, g1b), "repeat calls differ"
    d2, g2, _, _, b2 = once({"QDC_DYN": "35"})
    assert np.array_equal(g1, g2) and np.array_equal(b1, b2), "two circuits differ"
    d3, g3, _, _, _ = once({"QDC_DYN": "100"})
    tol = 1e-5 if prec == "f32" else 1e-12
    assert F.normrel(g3, g1) <= tol and F.normrel(d3, d1) <= tol
    print(f"[dyn] {prec} n={n}: static-only vs dynamic tail, grads {F.normrel(g3, g1):.2e}")


@pytest.mark.parametrize("prec,case", [("f32", "layered14"), ("f32", "random14"), ("f32", "layered18"),
                                       ("f64", "layered14"), ("f64", "random14")])
def test_specialized_passes_equal_interpreted(prec, case):
    """Passes compiled per pass program (csrc/qdc_spec.hpp, qdc_jit.hpp: straight-line stages,
    compile-time slot cases and relayout descriptors; two-state reverse passes and one-state
    forward passes; QDC_SPEC=2 forces them at any size, 0 keeps the interpreted k_rw / k_rq)
    run the same stage arithmetic in the same order as the interpreted kernels: densities,
    gradients and both states are bit-identical, and within the floors of the oracle."""
    import quantum_differentiable_circuit as q
    kind, n = case[:-2], int(case[-2:])
    if kind == "layered":
        ins, var = O.layered_circuit(n, 4, seed=31)
        const, psi0 = [], None
    else:
        ins, const, var = O.random_circuit(n, 160, seed=300 + n, density_every=3)
        psi0 = O.random_state(np.random.default_rng(n + 1), n)
    fl = F.Floor(prec, n, ins, const, var, psi0=psi0, run=False)
    out = {}
    for mode in ("0", "2"):
        c = build_env(prec, n, ins, {"QDC_SPEC": mode, "QDC_SPEC_MAX": 400})
        if psi0 is not None:
            c.set_state_from_vector(fl.psi0)
        launched = q.jit_stats(prec)["launched"]
        d = c.forward(fl.const, fl.var)
        g = c.backward(fl.cots, fl.const, fl.var)
        c.synchronize()
        ran = q.jit_stats(prec)["launched"] - launched
        # the forced mode really ran specialized kernels (a failed compile would fall back to
        # the interpreted ones and make this comparison vacuous); mode 0 none
        assert (ran > 0) == (mode == "2"), (mode, ran, q.jit_stats(prec))
        flat = lambda xs: np.concatenate([np.asarray(x).reshape(-1) for x in xs])
        out[mode] = (flat(d), flat(g), np.asarray(c.get_state(0)), np.asarray(c.get_state(2)))
        what = f"{prec} {case} spec={mode} "
        fl.check("grads", g, what)
        fl.check("uncomputed", out[mode][2], what)
    # (grads are per-gate arrays of different shapes: compared flattened)
    # f32: bit-identical (the stages' packed FMAs are explicit).  f64: the scalar complex
    # products a.x * b.x - a.y * b.y have two FMA contractions, and the compiler may pick the
    # other one in straight-line code than in the interpreted loop: within 1e-14 relative.
    for k, name in enumerate(("densities", "grads", "fwd", "bwd")):
        a0, a2 = out["0"][k], out["2"][k]
        if prec == "f32":
            assert np.array_equal(a0, a2), f"{prec} {case}: specialized {name} differ"
        else:
            rel = np.linalg.norm(a2 - a0) / max(np.linalg.norm(a0), 1e-300)
            print(f"[spec] {prec} {case} {name}: relative difference {rel:.2e}")
            assert rel <= 1e-14, f"{prec} {case}: specialized {name} differ by {rel:.2e}"
    print(f"[spec] {prec} {case}: specialized passes match the interpreted kernels")


ABL_LIB = Path(__file__).resolve().parent.parent / "differentiable-quantum-circuit-cuda_amd" / "lib-abl"


@pytest.mark.skipif(not (ABL_LIB / "libqdc_f32.so").exists(), reason="ablation build not built")
def test_ablation_library_kernels_never_reach_production(tmp_path):
    """The timing-only ablation library (csrc/Makefile `abl`, QDC_RQ_ABL=1: no stage math, wrong
    results) runs a circuit with specialized passes into a cache directory; the production
    library then runs the same circuit against the same directory.  The build fingerprint in
    the kernel names (qdc_jit.hpp) keeps the ablation kernels out: the production process
    compiles and launches its own, and its results are within the oracle's floors."""
    import json
    import subprocess
    import sys
    n = 14
    ins, var = O.layered_circuit(n, 3, seed=51)
    fl = F.Floor("f32", n, ins, [], var, run=False)
    np.save(tmp_path / "cots.npy", np.stack([np.asarray(x).reshape(-1) for x in fl.cots]))
    root = Path(__file__).resolve().parent.parent
    code = f"""
import json, sys
import numpy as np
sys.path[:0] = [{str(root)!r}, {str(root / 'differentiable-quantum-circuit-cuda_amd')!r}]
import quantum_differentiable_circuit as q
from oracle import oracle as O
ins, var = O.layered_circuit({n}, 3, seed=51)
c = q.circuit_class("f32")({n})
for kind, pos in ins:
    c._push(kind, *pos)
vg = [np.ascontiguousarray(g, dtype=np.complex64) for g in var]
d = c.forward([], vg)
cots = [np.ascontiguousarray(x.reshape(2, 2)) for x in np.load({str(tmp_path / 'cots.npy')!r})]
g = c.backward(cots, [], vg)
c.synchronize()
np.save(sys.argv[1] + "_d.npy", np.concatenate([np.asarray(x).reshape(-1) for x in d]))
np.save(sys.argv[1] + "_g.npy", np.concatenate([np.asarray(x).reshape(-1) for x in g]))
print(json.dumps(q.jit_stats("f32")))
"""
    (tmp_path / "jit").mkdir(mode=0o700)
    stats = {}
    for tag, libdir in (("abl", ABL_LIB), ("prod", None)):
        env = dict(os.environ, QDC_SPEC="2", QDC_JIT_DIR=str(tmp_path / "jit"))
        env.pop("QDC_LIB_DIR", None)
        if libdir is not None:
            env["QDC_LIB_DIR"] = str(libdir)
        r = subprocess.run([sys.executable, "-c", code, str(tmp_path / tag)], env=env,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        stats[tag] = json.loads(r.stdout.strip().splitlines()[-1])
        print(f"[abl] {tag}: {stats[tag]}")
    for tag in ("abl", "prod"):
        assert stats[tag]["enabled"] and stats[tag]["compiled"] > 0 and stats[tag]["launched"] > 0
    fl.check("forward", np.load(tmp_path / "prod_d.npy"), "ablation-then-production ")
    grads = np.load(tmp_path / "prod_g.npy")
    fl.check("grads", grads, "ablation-then-production ")
    assert F.normrel(np.load(tmp_path / "abl_g.npy"), grads) > 1e-3, "the ablation build computed real gradients"


def _diag_cots(seed):
    """random complex diagonal cotangents (Q1 and Q2 densities): the diagonal-injection path"""
    rng = np.random.default_rng(seed)

    def cots(dens, dt):
        return [np.ascontiguousarray(np.diag(rng.standard_normal(d.shape[0])
                                             + 1j * rng.standard_normal(d.shape[0])).astype(dt))
                for d in dens]
    return cots


@pytest.mark.parametrize("prec", ["f32", "f64"])
@pytest.mark.parametrize("case", ["layered", "random", "sharded"])
def test_diagonal_injections_equal_general(prec, case):
    """Runs of cotangent injections whose cotangents are all diagonal (Z-basis observables) are one
    elementwise pass (k_diag_inject: b (+)= 2 conj(f) D, D summed over the run's densities) instead
    of the LDS injection passes; QDC_DIAG_INJECT=0 keeps the general path.  Both match the oracle's
    floors and each other: densities at the end (layered: the run starts bwd), interleaved with
    gates (random: Q1 and Q2 densities, runs accumulating into an existing bwd), and on 4 local
    shards."""
    import quantum_differentiable_circuit as q
    n = 14 if case != "random" else 12
    if case == "random":
        ins, const, var = O.random_circuit(n, 160, seed=77, density_every=20)
        psi0 = O.random_state(np.random.default_rng(5), n)
    else:
        ins, var = O.layered_circuit(n, 3, seed=61)
        const, psi0 = [], None
    fl = F.Floor(prec, n, ins, const, var, psi0=psi0, cots=_diag_cots(3), run=False)
    kw = {"local_shards": 4} if case == "sharded" else {}
    out = {}
    for mode in ("0", "1"):
        c = build_env(prec, n, ins, {"QDC_DIAG_INJECT": mode}) if not kw else None
        if kw:
            old = os.environ.get("QDC_DIAG_INJECT")
            os.environ["QDC_DIAG_INJECT"] = mode
            try:
                c = q.circuit_class(prec)(n, **kw)
            finally:
                if old is None:
                    del os.environ["QDC_DIAG_INJECT"]
                else:
                    os.environ["QDC_DIAG_INJECT"] = old
            for kind, pos in ins:
                c._push(kind, *pos)
        if psi0 is not None:
            c.set_state_from_vector(fl.psi0)
        c.forward(fl.const, fl.var)
        c.profile(True)
        g = c.backward(fl.cots, fl.const, fl.var)
        stats = c.profile_collect()
        what = f"diag-inject {case} {prec} mode={mode} "
        fl.check("grads", g, what)
        if case != "sharded":
            fl.check("bwd", c.get_state(2), what)
        assert ("inject_diag" in stats) == (mode == "1"), sorted(stats)
        out[mode] = g
    F.check_pair(prec, out["1"], out["0"], fl.floor["grads"], f"diag-inject {case} {prec} on vs off grads")


@pytest.mark.parametrize("prec", ["f32", "f64"])
@pytest.mark.parametrize("n", [16, 20])
def test_density_only_passes_and_split(monkeypatch, prec, n):
    """Round 6: forward passes hold gates or densities, not both (QDC_DENS_SPLIT), so the last
    gates stay register-resident, and density-only passes of one-qubit densities run on k_dens1
    (QDC_DENS1: register partial sums across a block's tiles) — against the floors, and against
    the round-5 schedule (mixed passes, k_fused's per-tile reductions) within 8x the floor; with
    q1 and q2 densities mid-circuit too (mixed-kind density passes stay on k_fused)."""
    ins, var = O.layered_circuit(n, 3, seed=11)
    cut = len(ins) // 2
    ins = ins[:cut] + [(O.DIFF_Q1_DENSITY, (q,)) for q in (0, 5, n - 1)] + \
        [(O.DIFF_Q2_DENSITY, (n - 2, 3))] + ins[cut:]
    fl = F.Floor(prec, n, ins, [], var, run=False)
    res = {}
    for new in (False, True):
        for k in ("QDC_DENS_SPLIT", "QDC_DENS1"):
            if new:
                monkeypatch.delenv(k, raising=False)
            else:
                monkeypatch.setenv(k, "0")
        c = build(prec, n, ins, 1)
        c.profile(True)
        what = f"density passes n={n} {prec} {'split + k_dens1' if new else 'round 5'} "
        d = c.forward([], fl.var)
        g = c.backward(fl.cots, [], fl.var)
        fl.check("forward", d, what)
        fl.check("grads", g, what)
        res[new] = (d, g, c.profile_collect())
    F.check_pair(prec, res[True][0], res[False][0], fl.floor["forward"], f"n={n} {prec} densities new vs round 5")
    F.check_pair(prec, res[True][1], res[False][1], fl.floor["grads"], f"n={n} {prec} grads new vs round 5")
    assert res[True][2]["fused_density"]["launches"] >= 1, sorted(res[True][2])

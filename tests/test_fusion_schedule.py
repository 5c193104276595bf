"""The fused-pass scheduler on CPU (qdc_fusion_schedule: the runtime's own host code).

1. Structural invariants on random circuits over every gate kind, with densities, for the
   forward and the reverse sweep:
   * every plan op runs exactly once;
   * per qubit, program order is kept;
   * a density / injection ("meas") and a "sensitive" gate never swap: in the forward, a
     non-NonU gate is sensitive when its matrix is not unitary; in the reverse sweep, variable
     and NonU gates are;
   * in the reverse sweep, a non-NonU gate with a non-unitary matrix and a variable gate never
     swap;
   * every op of a fused pass lies in its tile (lc contiguous chunk bits, >= lcmin, plus h row
     bits, lc + h = log2 tile);
   * a stage spans at most two qubits, and a meas op is a stage of its own;
   * reverse-sweep passes are all injections or no injection, and never span the first one.
2. Semantics: the schedule's execution order, replayed with the oracle's primitives
   (oracle/oracle.py, restating src/circuit.rs:164-429), gives the sequential densities and
   gradients (f64, 1e-12) - including matrices that are not unitary on unitary kinds.
"""
import numpy as np
import pytest

from oracle import oracle as O

Q1 = (O.CONST_Q1, O.CONST_Q1_NONU, O.VAR_Q1, O.VAR_Q1_NONU)
Q2 = (O.CONST_Q2, O.VAR_Q2, O.CONST_Q2_NONU, O.VAR_Q2_NONU)
DIAG = (O.CONST_Q2_DIAG, O.VAR_Q2_DIAG)
CONST = (O.CONST_Q1, O.CONST_Q1_NONU, O.CONST_Q2, O.CONST_Q2_NONU, O.CONST_Q2_DIAG)
NONU = (O.CONST_Q1_NONU, O.VAR_Q1_NONU, O.CONST_Q2_NONU, O.VAR_Q2_NONU)
DENS = (O.Q1_DENSITY, O.Q2_DENSITY, O.DIFF_Q1_DENSITY, O.DIFF_Q2_DENSITY)
LV = {"f32": 1, "f64": 0}
T = {1: 11, 2: 10}  # log2 tile chunks: one-state (forward) / two-state (reverse)


def unitary_error(g, kind):
    if kind in DIAG:
        return np.abs(np.abs(g) ** 2 - 1).max()
    r = 2 if kind in Q1 else 4
    m = np.asarray(g).reshape(r, r)
    return np.abs(m.conj().T @ m - np.eye(r)).max()


def make(n, seed, perturb=0.0):
    ins, const, var = O.random_circuit(n, 150, seed=seed, density_every=4)
    ins = ins[:30] + [(O.Q1_DENSITY, (2,)), (O.Q2_DENSITY, (n - 1, 1))] + ins[30:]
    if perturb:
        rng = np.random.default_rng(seed)
        var = [g + perturb * (rng.standard_normal(g.shape) + 1j * rng.standard_normal(g.shape))
               for g in var]
    gates, ci, vi = {}, 0, 0
    for i, (k, _) in enumerate(ins):
        if k in CONST:
            gates[i], ci = const[ci], ci + 1
        elif k not in DENS:
            gates[i], vi = var[vi], vi + 1
    sens = [int(i in gates and unitary_error(gates[i], ins[i][0]) > 1e-13) for i in range(len(ins))]
    return ins, const, var, gates, sens


def schedule(n, ins, mode, sens, prec):
    import quantum_differentiable_circuit as q
    instr = [(k, *p) for k, p in ins]
    return q.fusion_schedule(n, instr, mode, fwd_sens=sens, precision=prec)


def qubits(ins, op):
    k, p = ins[op["instr"]]
    return set(p)


def check_invariants(n, ins, sens, mode, prec, ops, items, permuted=False, tbits=None):
    backward = mode == 2
    order = [i for it in items for st in it["stages"] for i in st]
    assert sorted(order) == list(range(len(ops)))
    pos = {i: k for k, i in enumerate(order)}
    kinds = [ins[o["instr"]][0] for o in ops]
    meas = [k in DENS for k in kinds]
    if backward:
        sensitive = [k in NONU or (k not in DENS and k not in CONST) for k in kinds]
    else:
        sensitive = [k not in DENS and (k in NONU or sens[o["instr"]]) for k, o in zip(kinds, ops)]
    # reverse sweep: a non-NonU gate with a non-unitary matrix keeps its order relative to
    # variable gates (their gradients see B^T A != I otherwise)
    isvar = [backward and k not in DENS and k not in CONST for k in kinds]
    inexact = [backward and k not in DENS and k not in NONU and bool(sens[o["instr"]])
               for k, o in zip(kinds, ops)]
    for a in range(len(ops)):
        for b in range(a + 1, len(ops)):
            share = qubits(ins, ops[a]) & qubits(ins, ops[b])
            clash = (meas[a] and sensitive[b]) or (sensitive[a] and meas[b]) or \
                (inexact[a] and isvar[b]) or (isvar[a] and inexact[b])
            if share or clash:
                assert pos[a] < pos[b], (a, b, ops[a], ops[b])
    first_inject = next((i for i, m in enumerate(meas) if m), len(ops)) if backward else len(ops)
    tbits = tbits or T[2 if backward else 1]
    for it in items:
        if it["type"] != 2:
            assert len(it["stages"]) == 1 and len(it["stages"][0]) == 1
            continue
        assert it["lc"] >= 3 and it["lc"] + it["h"] == tbits
        tile = set(range(LV[prec] + it["lc"])) | {LV[prec] + c for c in it["hb"]}
        members = [i for st in it["stages"] for i in st]
        for i in members:  # (permuting passes move qubits: tiles are in the permuted layout)
            assert permuted or qubits(ins, ops[i]) <= tile | set(range(LV[prec])), (i, it)
        if backward:
            assert len({meas[i] for i in members}) == 1
            assert len({i >= first_inject for i in members}) == 1
        for st in it["stages"]:
            qs = set().union(*(qubits(ins, ops[i]) for i in st))
            assert len(qs) <= 2
            if any(meas[i] for i in st):
                assert len(st) == 1


@pytest.mark.parametrize("prec", ["f32", "f64"])
@pytest.mark.parametrize("n,seed,perturb", [(14, 1, 0.0), (17, 2, 1e-3), (24, 3, 0.0)])
def test_schedule_invariants(prec, n, seed, perturb):
    ins, const, var, gates, sens = make(n, seed, perturb)
    for mode in (0, 1, 2):
        ops, items = schedule(n, ins, mode, sens, prec)
        check_invariants(n, ins, sens, mode, prec, ops, items)
        assert any(it["type"] == 2 for it in items)


def replay(n, ins, ops, items, gates, psi0, cot_fn):
    """Forward then reverse sweep in the schedule's execution order (oracle primitives)."""
    dens = {}
    state = psi0.copy()
    f_ops, f_items = ops["fwd"], items["fwd"]
    for it in f_items:
        for st in it["stages"]:
            for i in st:
                k, p = ins[f_ops[i]["instr"]]
                idx = f_ops[i]["instr"]
                if k in (O.DIFF_Q1_DENSITY, O.Q1_DENSITY):
                    dens[idx] = O.get_q1_density(state, p[0]).reshape(2, 2)
                elif k in (O.DIFF_Q2_DENSITY, O.Q2_DENSITY):
                    dens[idx] = O.get_q2_density(state, *p).reshape(4, 4)
                elif k in Q1:
                    state = O.apply_q1_gate(state, gates[idx], p[0])
                elif k in Q2:
                    state = O.apply_q2_gate(state, gates[idx], *p)
                else:
                    state = O.apply_q2_gate_diag(state, gates[idx], *p)
    dlist = [dens[i] for i in sorted(dens) if ins[i][0] in (O.DIFF_Q1_DENSITY, O.DIFF_Q2_DENSITY)]
    cots = cot_fn(dlist)
    cot_of = dict(zip([i for i in sorted(dens) if ins[i][0] in (O.DIFF_Q1_DENSITY, O.DIFF_Q2_DENSITY)],
                      cots))
    bwd, grads = None, {}
    b_ops, b_items = ops["bwd"], items["bwd"]
    for it in b_items:
        for st in it["stages"]:
            for i in st:
                idx = b_ops[i]["instr"]
                k, p = ins[idx]
                if k in (O.DIFF_Q1_DENSITY, O.DIFF_Q2_DENSITY):
                    gt = O.transpose(cot_of[idx])
                    add = 2 * state.conj()
                    add = O.apply_q1_gate(add, gt, p[0]) if k == O.DIFF_Q1_DENSITY \
                        else O.apply_q2_gate(add, gt, *p)
                    bwd = add if bwd is None else bwd + add
                    continue
                g = gates[idx]
                unc = g.conj() if k in DIAG else (O.inverse(g) if k in NONU else O.conj_transpose(g))
                apply = (lambda s, m: O.apply_q1_gate(s, m, p[0])) if k in Q1 else \
                    (lambda s, m: O.apply_q2_gate(s, m, *p)) if k in Q2 else \
                    (lambda s, m: O.apply_q2_gate_diag(s, m, *p))
                state = apply(state, unc)
                if k not in CONST:
                    if bwd is None:
                        grads[idx] = np.zeros(16 if k in Q2 else 4, np.complex128)
                    elif k in Q1:
                        grads[idx] = O.get_q1_grad(state, bwd, p[0])
                    elif k in Q2:
                        grads[idx] = O.get_q2_grad(state, bwd, *p)
                    else:
                        grads[idx] = O.get_q2_grad_diag(state, bwd, *p)
                if bwd is not None:
                    bwd = apply(bwd, g if k in DIAG else O.transpose(g))
    return dlist, [grads[i] for i in sorted(grads)], state


@pytest.mark.parametrize("n,seed", [(14, 1), (24, 3)])
def test_permuting_schedule_invariants(monkeypatch, n, seed):
    """The f32 runtime's register-resident settings (QDC_SCHED_RQ: gate-only passes permute
    their tile's qubits, later positions are rewritten): ordering invariants still hold."""
    monkeypatch.setenv("QDC_SCHED_RQ", "1")
    ins, const, var, gates, sens = make(n, seed)
    for mode in (0, 1, 2):
        ops, items = schedule(n, ins, mode, sens, "f32")
        check_invariants(n, ins, sens, mode, "f32", ops, items, permuted=True)


@pytest.mark.parametrize("sched_rq", ["0", "1"])
@pytest.mark.parametrize("perturb", [0.0, 1e-3])
def test_schedule_replay_matches_sequential_oracle(monkeypatch, perturb, sched_rq):
    """Replaying the scheduled execution order (logical qubits) equals the sequential oracle;
    sched_rq = 1 uses the runtime's f32 permuting planner."""
    monkeypatch.setenv("QDC_SCHED_RQ", sched_rq)
    n = 12  # the smallest n whose tiles are full in both passes (f32: 2^11 chunks)
    ins, const, var, gates, sens = make(n, 11, perturb)
    ops, items = {}, {}
    ops["fwd"], items["fwd"] = schedule(n, ins, 1, sens, "f32")
    ops["bwd"], items["bwd"] = schedule(n, ins, 2, sens, "f32")
    assert sum(it["type"] == 2 for it in items["fwd"]) > 3
    assert sum(it["type"] == 2 for it in items["bwd"]) > 3
    psi0 = O.random_state(np.random.default_rng(4), n)
    o = O.OracleCircuit(n)
    for k, p in ins:
        o.add(k, *p)
    o.set_state_from_vector(psi0)
    want_d = o.forward(const, var)

    def cot_fn(d):
        return [c.conj() for c in O.tsallis_loss_and_cotangents(d)[1]]

    want_g = o.backward(cot_fn(want_d), const, var)
    got_d, got_g, final = replay(n, ins, ops, items, gates, psi0, cot_fn)
    assert len(got_d) == len(want_d) and len(got_g) == len(want_g)
    for a, b in zip(got_d, want_d):
        assert np.abs(a - b).max() < 1e-12
    ga, gb = np.concatenate(got_g), np.concatenate(want_g)
    assert np.abs(ga - gb).max() < 1e-11 * np.abs(gb).max()
    assert np.abs(final - o.state).max() < 1e-11


def mirrored(ops_f, items_f, ins):
    """The backward schedule QDC_MIRROR runs (qdc_circuit.hpp mirror_schedule): the forward's
    passes in reverse, stages and the ops in them reversed; a pass's trailing densities become
    the injections that open its reverse pass (one item).  Forward plan index i is backward plan
    index L - 1 - i (both plans hold the gates and differentiable densities)."""
    L = len(ops_f)
    items = []
    for it in reversed(items_f):
        stages = it["stages"]
        ng = len(stages)
        while ng and ins[ops_f[stages[ng - 1][0]]["instr"]][0] in DENS:
            ng -= 1
        if ng < len(stages):
            st = [[L - 1 - s[0]] for s in reversed(stages[ng:])]
            items.append(dict(it, type=2 if len(st) > 1 else 0, stages=st))
        if ng:
            st = [[L - 1 - i for i in reversed(s)] for s in reversed(stages[:ng])]
            items.append(dict(it, stages=st))
    return ops_f[::-1], items


@pytest.mark.parametrize("prec", ["f32", "f64"])
@pytest.mark.parametrize("sched_rq", ["0", "1"])
@pytest.mark.parametrize("n,seed,perturb", [(14, 1, 0.0), (17, 2, 1e-3), (24, 3, 0.0)])
def test_mirrored_schedule_invariants(monkeypatch, prec, sched_rq, n, seed, perturb):
    """QDC_MIRROR: the forward is scheduled on the two-state tile so that its passes run in
    reverse are a valid reverse sweep - the invariants of both directions hold, none spans the
    last differentiable density, and the Gamma
    stages (stages holding a variable gate) of a pass fit the 16 accumulators; a pass holds gate
    stages, then densities."""
    monkeypatch.setenv("QDC_SCHED_RQ", sched_rq)
    monkeypatch.setenv("QDC_SCHED_MIRROR", "1")
    ins, const, var, gates, sens = make(n, seed, perturb)
    ops_f, items_f = schedule(n, ins, 1, sens, prec)
    perm = sched_rq == "1"
    check_invariants(n, ins, sens, 1, prec, ops_f, items_f, permuted=perm, tbits=T[2])
    ops_b, items_b = mirrored(ops_f, items_f, ins)
    check_invariants(n, ins, sens, 2, prec, ops_b, items_b, permuted=perm, tbits=T[2])
    var_kinds = set(Q1 + Q2 + DIAG) - set(CONST)
    for it in items_f:
        if it["type"] != 2:
            continue
        meas = [ins[ops_f[st[0]]["instr"]][0] in DENS for st in it["stages"]]
        assert meas == sorted(meas)  # gate stages, then densities
        gst = sum(any(ins[ops_f[i]["instr"]][0] in var_kinds for i in st) for st in it["stages"])
        assert gst <= 16
    assert sum(it["type"] == 2 for it in items_f) > 3


@pytest.mark.parametrize("sched_rq", ["0", "1"])
def test_mirrored_schedule_replay_matches_sequential_oracle(monkeypatch, sched_rq):
    """The mirrored reverse sweep, replayed with the oracle's primitives, gives the sequential
    densities and gradients (non-unitary matrices on unitary kinds included)."""
    monkeypatch.setenv("QDC_SCHED_RQ", sched_rq)
    monkeypatch.setenv("QDC_SCHED_MIRROR", "1")
    n = 12
    ins, const, var, gates, sens = make(n, 11, 1e-3)
    ops, items = {}, {}
    ops["fwd"], items["fwd"] = schedule(n, ins, 1, sens, "f32")
    ops["bwd"], items["bwd"] = mirrored(ops["fwd"], items["fwd"], ins)
    assert sum(it["type"] == 2 for it in items["fwd"]) > 3
    psi0 = O.random_state(np.random.default_rng(5), n)
    o = O.OracleCircuit(n)
    for k, p in ins:
        o.add(k, *p)
    o.set_state_from_vector(psi0)
    want_d = o.forward(const, var)

    def cot_fn(d):
        return [c.conj() for c in O.tsallis_loss_and_cotangents(d)[1]]

    want_g = o.backward(cot_fn(want_d), const, var)
    got_d, got_g, final = replay(n, ins, ops, items, gates, psi0, cot_fn)
    for a, b in zip(got_d, want_d):
        assert np.abs(a - b).max() < 1e-12
    ga, gb = np.concatenate(got_g), np.concatenate(want_g)
    assert np.abs(ga - gb).max() < 1e-11 * np.abs(gb).max()
    assert np.abs(final - o.state).max() < 1e-11


@pytest.mark.parametrize("mirror", ["0", "1"])
def test_trailing_one_qubit_stages_join_the_next_pass(monkeypatch, mirror):
    """C2's generator at n = 28 (20 layers) on the runtime's f32 settings: a stage of one-qubit
    gates left at the end of a pass moves to the pass of its qubit's next two-qubit gate
    (defer_trailing_q1), so almost every one-qubit gate shares a two-qubit gate's stage — the
    minimum is one stage per two-qubit gate (540)."""
    from quantum_differentiable_circuit import workloads as W
    monkeypatch.setenv("QDC_SCHED_RQ", "1")
    monkeypatch.setenv("QDC_SCHED_MIRROR", mirror)
    n = 28
    ins, _ = W.layered_circuit(n, 20, 1)
    stages = {}
    for defer in ("0", "1"):
        monkeypatch.setenv("QDC_DEFER_Q1", defer)
        ops, items = schedule(n, ins, 2 if mirror == "0" else 1, [0] * len(ins), "f32")
        check_invariants(n, ins, [0] * len(ins), 2 if mirror == "0" else 1, "f32", ops, items,
                         permuted=True, tbits=T[2])
        stages[defer] = sum(1 for it in items if it["type"] == 2 for s in it["stages"]
                            if ins[ops[s[0]]["instr"]][0] not in DENS)
    assert stages["1"] <= 542 and stages["1"] <= stages["0"], stages

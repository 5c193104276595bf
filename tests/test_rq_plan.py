"""Register-layout plans of register-resident passes (qdc_rq_plan: the runtime's own host
planner, csrc/qdc_fusion.hpp rq_plan) on CPU.

A plan is valid when, replayed step by step:
  * the load and store layouts are HBM layouts (f32: slot 0 = tile bit 0, tile bits 1..3 are
    thread bits; f64, a 16-B chunk per amplitude: tile bits 0..2 are thread bits), and every
    layout holds 4 distinct tile bits;
  * every stage runs exactly once, after the stages it depends on;
  * a stage runs on the current layout with its qubits in the slots its slot case names
    (one-qubit: the slot of t1; two-qubit / diagonal: 8 * slot(t1) + slot(t2)).
The max-closure planner (default) must not need more relayouts in total than the greedy one
(QDC_RQ_MAXCL=0) on brickwork-like and random passes.
"""
import numpy as np
import pytest

Q1, Q2, DIAG = 0, 1, 2


def random_pass(rng, T, nst, brick=False):
    stages, masks = [], []
    for k in range(nst):
        if brick:
            a = int(rng.integers(0, T - 1))
            kind, t1, t2 = (Q1, a, a) if k % 3 == 0 else (Q2, a, a + 1)
        else:
            kind = int(rng.choice([Q1, Q2, DIAG]))
            if kind == Q1:
                t1 = t2 = int(rng.integers(0, T))
            else:
                t1, t2 = sorted(int(x) for x in rng.choice(T, 2, replace=False))
        stages.append((kind, t1, t2))
        masks.append((1 << t1) | (1 << t2))
    deps = [sum(1 << i for i in range(k) if masks[i] & masks[k]) for k in range(nst)]
    return stages, deps


def check_plan(T, stages, deps, plan, prec="f32", slots=4):
    load, steps, store = plan

    def hbm_ok(L):
        if prec == "f64":
            return not ({0, 1, 2} & set(L))
        return L[0] == 0 and not ({1, 2, 3} & set(L))

    assert hbm_ok(load) and hbm_ok(store), (load, store)
    cur, done, relayouts = list(load), set(), 0
    for s in steps:
        L = s["slots"]
        assert len(set(L)) == slots and all(q < T for q in L), L
        if s["relayout"]:
            cur, relayouts = list(L), relayouts + 1
            continue
        assert list(L) == cur
        j = s["stage"]
        kind, t1, t2 = stages[j]
        assert j not in done and all((deps[j] >> i) & 1 == 0 or i in done for i in range(j))
        if kind == Q1:
            assert cur[s["case"]] == t1
        else:
            assert cur[s["case"] // 8] == t1 and cur[s["case"] % 8] == t2
        done.add(j)
    assert done == set(range(len(stages)))
    assert cur == list(store)
    return relayouts


@pytest.mark.parametrize("prec,T,slots", [("f32", 11, 4), ("f32", 12, 4), ("f32", 11, 5),
                                           ("f64", 10, 4), ("f64", 11, 4)])
@pytest.mark.parametrize("brick", [False, True])
def test_rq_plan_valid_and_max_closure_not_worse(monkeypatch, prec, T, slots, brick):
    import quantum_differentiable_circuit as q
    rng = np.random.default_rng(T * 2 + brick)
    total = {"1": 0, "0": 0}
    for _ in range(120):
        stages, deps = random_pass(rng, T, int(rng.integers(1, 40)), brick)
        for mc in ("1", "0"):
            monkeypatch.setenv("QDC_RQ_MAXCL", mc)
            total[mc] += check_plan(T, stages, deps,
                                    q.rq_plan(T, stages, deps, precision=prec, slots=slots),
                                    prec, slots)
    assert total["1"] <= total["0"], total


@pytest.mark.parametrize("brick", [False, True])
def test_rq_plan_five_slots_fewer_relayouts(brick):
    """A fifth register slot (the one-wave two-state kernel's register-group bit) holds covers
    of 5 qubits: never more relayouts than 4 slots over a set of passes."""
    import quantum_differentiable_circuit as q
    rng = np.random.default_rng(7 + brick)
    total = {4: 0, 5: 0}
    for _ in range(120):
        stages, deps = random_pass(rng, 11, int(rng.integers(4, 40)), brick)
        for sl in (4, 5):
            total[sl] += check_plan(11, stages, deps,
                                    q.rq_plan(11, stages, deps, precision="f32", slots=sl),
                                    "f32", sl)
    print("relayouts 4 / 5 slots:", total)
    assert total[5] < total[4], total


@pytest.mark.parametrize("brick", [False, True])
def test_rq_plan_keep_slot_for_half_buffers(monkeypatch, brick):
    """rq_plan keep (QDC_RQ_KEEP; the runtime's one-wave five-slot passes): every relayout keeps
    one register slot's tile bit in the same slot, so the exchange runs in two rounds through
    half the LDS buffer (qdc_spec.hpp spec_xchg_half).  Plans stay valid; the cost in relayouts
    over a set of passes is printed and bounded."""
    import quantum_differentiable_circuit as q
    rng = np.random.default_rng(31 + brick)
    total = {"0": 0, "1": 0}
    for _ in range(120):
        stages, deps = random_pass(rng, 11, int(rng.integers(4, 40)), brick)
        for keep in ("0", "1"):
            monkeypatch.setenv("QDC_RQ_KEEP", keep)
            plan = q.rq_plan(11, stages, deps, precision="f32", slots=5)
            total[keep] += check_plan(11, stages, deps, plan, "f32", 5)
            if keep == "1":
                cur = list(plan[0])
                for s in plan[1]:
                    if s["relayout"]:
                        assert any(a == b for a, b in zip(cur, s["slots"])), (cur, s["slots"])
                        cur = list(s["slots"])
    print("relayouts without / with a kept slot:", total)
    assert total["1"] <= 1.5 * total["0"], total

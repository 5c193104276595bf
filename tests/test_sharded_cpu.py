"""The sharded-state path on CPU ranks (gloo, world size 2, 4 and 8).

Each rank executes the native planner's plans (qdc_plan, the same code the HIP runtime runs)
on a numpy shard of 2^(n-g) amplitudes: ops at the planned physical positions with the
oracle's primitives, REMAPs as the runtime performs them (pack the victim bits to the top,
then one all_to_all_single), densities and gradients as per-shard partials summed with an
all-reduce.  The results must equal the unsharded oracle (src/circuit.rs:164-429)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as O

Q1 = (O.CONST_Q1, O.CONST_Q1_NONU, O.VAR_Q1, O.VAR_Q1_NONU)
Q2 = (O.CONST_Q2, O.VAR_Q2, O.CONST_Q2_NONU, O.VAR_Q2_NONU)
DIAG = (O.CONST_Q2_DIAG, O.VAR_Q2_DIAG)
CONST = (O.CONST_Q1, O.CONST_Q1_NONU, O.CONST_Q2, O.CONST_Q2_NONU, O.CONST_Q2_DIAG)
NONU = (O.CONST_Q1_NONU, O.VAR_Q1_NONU, O.CONST_Q2_NONU, O.VAR_Q2_NONU)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def pack(shard, victims, nl):
    """dst[o] = src[expand(o)]: the runtime's k_pack (csrc/qdc_kernels.hpp)."""
    g = len(victims)
    low = nl - g
    o = np.arange(1 << nl)
    idx = o & ((1 << low) - 1)
    for v in victims:  # ascending zero insertion
        lo = idx & ((1 << v) - 1)
        idx = ((idx - lo) << 1) | lo
    j = o >> low
    for k, v in enumerate(victims):
        idx |= ((j >> k) & 1) << v
    return shard[idx]


def remap(shard, r, nl, world):
    send = pack(shard, r["victims"], nl) if r["pack"] else shard
    t = torch.from_numpy(np.ascontiguousarray(send)).view(torch.float64)
    out = torch.empty_like(t)
    dist.all_to_all_single(out, t)
    return out.view(torch.complex128).numpy().copy()


def unpack(shard, victims, nl):
    """The inverse of pack: dst[expand(o)] = src[o] (k_pack<true>)."""
    g = len(victims)
    low = nl - g
    o = np.arange(1 << nl)
    idx = o & ((1 << low) - 1)
    for v in victims:
        lo = idx & ((1 << v) - 1)
        idx = ((idx - lo) << 1) | lo
    j = o >> low
    for k, v in enumerate(victims):
        idx |= ((j >> k) & 1) << v
    out = np.empty_like(shard)
    out[idx] = shard
    return out


def unremap(shard, r, nl, world):
    """The runtime's unremap (csrc/qdc_circuit.hpp): the all-to-all, then the inverse pack."""
    t = torch.from_numpy(np.ascontiguousarray(shard)).view(torch.float64)
    out = torch.empty_like(t)
    dist.all_to_all_single(out, t)
    got = out.view(torch.complex128).numpy().copy()
    return unpack(got, r["victims"], nl) if r["pack"] else got


def allreduce(x):
    t = torch.from_numpy(np.ascontiguousarray(np.asarray(x, np.complex128))).view(torch.float64)
    dist.all_reduce(t)
    return t.view(torch.complex128).numpy().copy()


def apply(shard, kind, p2, p1, g):
    if kind in Q1:
        return O.apply_q1_gate(shard, g, p2)
    if kind in Q2:
        return O.apply_q2_gate(shard, g, p2, p1)
    return O.apply_q2_gate_diag(shard, g, p2, p1)


def run_sharded(n, world, rank, ins, const, var, psi0, cot_fn, mirror=False):
    import quantum_differentiable_circuit as q
    g = world.bit_length() - 1
    nl = n - g
    instr = [(k, *p) for k, p in ins]
    shard = psi0[rank << nl:(rank + 1) << nl].astype(np.complex128).copy()
    # forward (Circuit::forward): gates + Diff densities; mirrored: the plan whose reverse, with
    # every remap undone, is the backward's (the runtime's mirrored reverse sweeps)
    ops, phys_end = q.plan(n, world, instr, mode=3 if mirror else 1, precision="f64")
    fwd_ops = ops
    kinds = [k for k, _ in ins]
    gidx, ci, vi = {}, 0, 0
    for i, k in enumerate(kinds):
        if k in CONST:
            gidx[i], ci = const[ci], ci + 1
        elif k not in (O.Q1_DENSITY, O.Q2_DENSITY, O.DIFF_Q1_DENSITY, O.DIFF_Q2_DENSITY):
            gidx[i], vi = var[vi], vi + 1
    # the planner may run ops out of program order (commuting ones): densities and
    # cotangents are keyed by instruction, as in the runtime
    dens = {}
    nremap = 0
    for op in ops:
        if op["type"] == "remap":
            shard = remap(shard, op, nl, world)
            nremap += 1
            continue
        k = kinds[op["instr"]]
        if k == O.DIFF_Q1_DENSITY:
            dens[op["instr"]] = O.get_q1_density(shard, op["pos2"])
        elif k == O.DIFF_Q2_DENSITY:
            dens[op["instr"]] = O.get_q2_density(shard, op["pos2"], op["pos1"])
        else:
            shard = apply(shard, k, op["pos2"], op["pos1"], gidx[op["instr"]])
    order = sorted(dens)
    dens = [allreduce(dens[i]).reshape(int(np.sqrt(dens[i].size)), -1) for i in order]
    cot_of = dict(zip(order, cot_fn(dens)))
    # backward (Circuit::backward): reverse order, starting from the forward's final layout
    if mirror:
        ops = [dict(o, undo=True) for o in reversed(fwd_ops)]
    else:
        ops, _ = q.plan(n, world, instr, mode=2, start_phys=phys_end, precision="f64")
    bwd = None
    grads = {}
    for op in ops:
        if op["type"] == "remap":
            move = unremap if op.get("undo") else remap
            shard = move(shard, op, nl, world)
            if bwd is not None:
                bwd = move(bwd, op, nl, world)
            nremap += 1
            continue
        i = op["instr"]
        k = kinds[i]
        p2, p1 = op["pos2"], op["pos1"]
        if k in (O.DIFF_Q1_DENSITY, O.DIFF_Q2_DENSITY):
            add = 2 * shard.conj()
            gt = O.transpose(cot_of[i])
            add = O.apply_q1_gate(add, gt, p2) if k == O.DIFF_Q1_DENSITY else O.apply_q2_gate(add, gt, p2, p1)
            bwd = add if bwd is None else bwd + add
            continue
        gate = gidx[i]
        unc = gate.conj() if k in DIAG else (O.inverse(gate) if k in NONU else O.conj_transpose(gate))
        shard = apply(shard, k, p2, p1, unc)
        if bwd is None:
            if k not in CONST:
                grads[i] = np.zeros(16 if k in Q2 else 4, np.complex128)
            continue
        if k not in CONST:
            if k in Q1:
                grads[i] = O.get_q1_grad(shard, bwd, p2)
            elif k in Q2:
                grads[i] = O.get_q2_grad(shard, bwd, p2, p1)
            else:
                grads[i] = O.get_q2_grad_diag(shard, bwd, p2, p1)
        bwd = apply(bwd, k, p2, p1, gate if k in DIAG else O.transpose(gate))
    grads = [allreduce(grads[i]) for i in sorted(grads)]
    if mirror:  # every remap undone: the uncomputed shard is back in the identity layout
        assert np.abs(shard - psi0[rank << nl:(rank + 1) << nl]).max() < 1e-10
    return dens, grads, nremap


def worker(rank, world, port, case, q_out):
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        n, ins, const, var, psi0, cot_fn = make_case(case)
        dens, grads, nremap = run_sharded(n, world, rank, ins, const, var, psi0, cot_fn,
                                          mirror=case.endswith("_mirror"))
        q_out.put((rank, dens, grads, nremap, None))
    except Exception as e:  # noqa: BLE001
        import traceback
        q_out.put((rank, None, None, 0, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def tsallis_cots(dens):
    return [c.conj() for c in O.tsallis_loss_and_cotangents(dens)[1]]


def sz_cots(dens):
    return [np.diag([1.0, -1.0]).astype(np.complex128) for _ in dens]


def make_case(case):
    case = case.removesuffix("_mirror")
    if case == "autodiff":
        n = 9
        ins, const, var, _ = O.autodiff_circuit(n, 2, seed=5)
        psi0 = O.random_state(np.random.default_rng(3), n)
        return n, ins, const, var, psi0, tsallis_cots
    n = 10  # brickwork whose gates straddle the shard boundary in every layer
    ins, var = O.layered_circuit(n, 3, seed=30)
    psi0 = np.zeros(1 << n, np.complex128)
    psi0[0] = 1
    return n, ins, [], var, psi0, sz_cots


CASES = ["autodiff", "layered", "autodiff_mirror", "layered_mirror"]


@pytest.mark.parametrize("world,case", [(w, c) for w in (2, 4) for c in CASES] +
                         [(8, "autodiff_mirror"), (8, "layered_mirror")])
def test_sharded_plan_execution_matches_oracle(world, case):
    """`*_mirror`: the mirrored forward plan (qdc_plan mode 3) and, as the backward, that plan
    reversed with every remap undone (all-to-all, then the inverse pack) — the schedule of the
    runtime's mirrored reverse sweeps on sharded circuits.  World 8: the 8-GPU configuration's
    rank count (three rank bits, gloo ranks on CPU), in the mirrored schedule the runtime runs."""
    ctx = mp.get_context("spawn")
    q_out = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, case, q_out)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q_out.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[4] is None, r[4]
    n, ins, const, var, psi0, cot_fn = make_case(case)
    o = O.OracleCircuit(n)
    for k, pos in ins:
        o.add(k, *pos)
    o.set_state_from_vector(psi0)
    dens = o.forward(const, var)
    grads = o.backward(cot_fn(dens), const, var)
    for rank, d, g, nremap, _ in res:
        assert nremap > 0, "the case must exercise remaps"
        for a, b in zip(d, dens):
            assert np.abs(a - b).max() < 1e-12
        assert np.abs(np.concatenate(g) - np.concatenate(grads)).max() < 1e-11 * np.abs(np.concatenate(grads)).max()


def test_planner_keeps_op_qubits_local():
    import quantum_differentiable_circuit as q
    n, world = 12, 8
    ins, var = O.layered_circuit(n, 2, seed=1)
    instr = [(k, *p) for k, p in ins]
    ops, end = q.plan(n, world, instr, mode=1, precision="f32")
    phys = list(range(n))
    g = 3
    for op in ops:
        if op["type"] == "remap":
            v = op["victims"]
            assert len(v) == g and all(1 <= x < n - g for x in v) and v == sorted(v)
            # replay the map update
            L = n - g
            npos = {}
            c = 0
            for p in range(L):
                if p not in v:
                    npos[p] = c
                    c += 1
            for j, x in enumerate(v):
                npos[x] = L + j
            for i in range(g):
                npos[L + i] = L - g + i
            phys = [npos[p] for p in phys]
        else:
            k, a = instr[op["instr"]][0], instr[op["instr"]][1]
            assert op["pos2"] == phys[a] < n - g
            if k not in (O.CONST_Q1, O.CONST_Q1_NONU, O.VAR_Q1, O.VAR_Q1_NONU, O.Q1_DENSITY,
                         O.DIFF_Q1_DENSITY):
                assert op["pos1"] == phys[instr[op["instr"]][2]] < n - g
    assert phys == end
    # single rank: never a remap
    ops1, end1 = q.plan(n, 1, instr, mode=1, precision="f32")
    assert all(o["type"] == "op" for o in ops1) and end1 == list(range(n))


def test_unpermute():
    from quantum_differentiable_circuit import unpermute
    rng = np.random.default_rng(0)
    n = 5
    psi = rng.standard_normal(1 << n)
    phys = [3, 0, 4, 1, 2]
    # build the physical array: physical index bit phys[q] = logical bit q
    physical = np.empty_like(psi)
    for i in range(1 << n):
        pi = sum(((i >> q) & 1) << phys[q] for q in range(n))
        physical[pi] = psi[i]
    assert np.array_equal(unpermute(physical, phys), psi)


def _id_worker(rank, path, q_out):
    from quantum_differentiable_circuit.distributed import exchange_id
    raw = exchange_id(rank, path, lambda: bytes(range(128)), timeout=60)
    q_out.put((rank, raw))


def test_rccl_id_file_exchange(tmp_path):
    """The torch-free RCCL bootstrap (distributed.exchange_id): rank 0 publishes the 128-byte
    id atomically, every other rank reads exactly it."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q_out = ctx.Queue()
    path = tmp_path / "nccl.id"
    ps = [ctx.Process(target=_id_worker, args=(r, path, q_out)) for r in (3, 2, 1, 0)]
    for p in ps:
        p.start()
    got = dict(q_out.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert all(v == bytes(range(128)) for v in got.values()) and len(got) == 4


def test_rccl_id_file_rejects_stale(tmp_path):
    """An id file left by an earlier launch (rank 0 died before removing it) carries that
    launch's rank-0 start time: a reader of this launch keeps polling instead of taking it, and
    takes the fresh file once this launch's rank 0 writes it."""
    import struct
    import threading
    from quantum_differentiable_circuit.distributed import exchange_id
    path = tmp_path / "nccl.id"
    now = 1.0e9
    path.write_bytes(bytes([7] * 128) + struct.pack("<d", now - 3600.0))  # stale, an hour old
    got = {}

    def reader():
        got["raw"] = exchange_id(1, path, None, timeout=30, start=now + 1.0)

    t = threading.Thread(target=reader)
    t.start()
    t.join(timeout=0.5)
    assert t.is_alive() and "raw" not in got  # still polling: the stale id was rejected
    exchange_id(0, path, lambda: bytes(range(128)), start=now)
    t.join(timeout=30)
    assert got["raw"] == bytes(range(128))


def _check_schedule(n, world, ins, precision="f32"):
    import ctypes as C
    from quantum_differentiable_circuit import _native
    lib = _native.load(precision)
    m = len(ins)
    kinds = (C.c_int * m)(*[k for k, _ in ins])
    a = (C.c_uint * m)(*[p[0] for _, p in ins])
    b = (C.c_uint * m)(*[p[1] if len(p) > 1 else 0 for _, p in ins])
    items, swaps = C.c_size_t(0), C.c_size_t(0)
    err = lib.qdc_check_schedule(n, world, kinds, a, b, m, C.byref(items), C.byref(swaps))
    assert not err, err.decode()
    return items.value, swaps.value


@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("case", ["layered", "brickwall", "random"])
def test_permuting_passes_on_sharded_schedules(world, case, monkeypatch):
    """Permuting passes on sharded circuits (qdc_fusion.hpp relabel_remap): replaying the layout
    through the runtime's own forward schedule, every op finds its qubits where the plan puts
    them and every remap's victims stay local and ascending; the permuting schedule needs fewer
    items than fixed layouts (QDC_RQ_PERM_SHARD=0)."""
    from quantum_differentiable_circuit import workloads as W
    n = 22
    if case == "layered":
        ins, _ = W.layered_circuit(n, 6, 24)
    elif case == "brickwall":
        ins, _ = W.brickwall_circuit(n, 12, 30)
    else:
        ins, _ = W.deep_random_circuit(n, 1500, 33)
    items, swaps = _check_schedule(n, world, ins)
    monkeypatch.setenv("QDC_RQ_PERM_SHARD", "0")
    items0, swaps0 = _check_schedule(n, world, ins)
    print(f"[perm] {case} world={world}: {items} items ({swaps} swaps) vs {items0} fixed ({swaps0})")
    if world > 1:
        assert swaps0 == 0
    assert swaps > 0 and items <= items0

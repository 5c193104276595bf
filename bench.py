#!/usr/bin/env python3
"""Headline benchmark: forward + backward gate applications per second of a differentiable
state-vector circuit on MI355X (BASELINE.json metric), with the HBM roofline of the dominant
kernel and the CPU baseline (the C/OpenMP restatement of the reference kernels) beside it.

Workload (SURVEY.md §8d, config C2's generator at the metric's target size): n = 28 qubits, f32,
L = 20 layers of [Haar 1-qubit variable gate on every qubit; Haar 2-qubit variable gates on
(i+1, i) for even i, then odd i], DiffQ1Density on every qubit, loss sum_q Re tr(rho_q sigma_z).
One step = Circuit.forward (all densities to the host) + Circuit.backward (all gate gradients
to the host), i.e. one loss-and-gradient call as in example_vqse_ising.py:107-133.

value = gates x steps / wall time (every gate is applied once forward and once in the fused
reverse sweep); inputs are resident in HBM before the timed region (gate matrices are 16-256 B
host arrays passed per call, as in the reference API).

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N, torch only as the launcher):
strong scaling — the SAME
n-qubit state is sharded over the N GPUs by its high qubits; gates on a global
qubit trigger a remap (pack + one RCCL all-to-all over xGMI), densities and gradients are
all-reduced.  value = the circuit's gates x steps / (max over ranks of the wall time).
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "differentiable-quantum-circuit-cuda_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md, chip-level parameters)
VALU_PEAK_TFLOPS = {"f32": 157.3, "f64": 78.6}  # vector peak (MI355X_MICROARCH.md; packed f32)
XGMI_LINK_GBS = 153.0  # one xGMI link of MI355X, per direction (7 point-to-point links per GPU)


class heartbeat:
    """A progress line on stderr every `every` s while a long silent phase runs (the CPU
    baseline's whole-step call takes minutes; a run that prints nothing for 3 minutes is taken
    to be hung)."""

    def __init__(self, label, every=30.0):
        import threading
        self.label, self.every, self.stop = label, every, threading.Event()
        self.t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        t0 = time.perf_counter()
        while not self.stop.wait(self.every):
            print(f"[bench] {self.label}: {time.perf_counter() - t0:.0f} s", file=sys.stderr,
                  flush=True)

    def __enter__(self):
        self.t.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        self.t.join()
        return False


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS),
                    help="BASELINE.json config: c2 layered random circuit (configs[1] generator, "
                         "the headline), c4 brickwall (configs[3]), c5 deep random (configs[4])")
    ap.add_argument("--qubits", type=int, default=None, help="default: the workload's n")
    ap.add_argument("--layers", type=int, default=None,
                    help="layers (c2, c4) or gates (c5); default: the workload's")
    ap.add_argument("--precision", default="f32", choices=["f32", "f64"])
    ap.add_argument("--seed", type=int, default=None, help="default: the workload's")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--local-shards", type=int, default=None,
                    help="rehearse the sharded data path on one GPU (G shards, device copies in "
                         "place of the RCCL all-to-all); not a multi-GPU measurement")
    ap.add_argument("--local-streams", type=int, default=None,
                    help="rehearse the single-process multi-GPU path on one GPU: G shards, each "
                         "on its own stream of device 0 (event-ordered copies in place of RCCL)")
    ap.add_argument("--no-gate-sample", action="store_true",
                    help="skip the single-gate (fusion off) kernel sweep and the other auxiliary samples")
    ap.add_argument("--cpu-layers", type=int, default=None,
                    help="layers of the C2 circuit the CPU baseline's headline call runs "
                         "(default: the GPU step's, i.e. the whole step)")
    ap.add_argument("--cpu-qubits", type=int, default=None)
    ap.add_argument("--cpu-c3-max-s", type=float, default=120.0,
                    help="time one whole C3 call on the CPU when its projection is below this")
    ap.add_argument("--pmc", default=None, help="JSON with PMC-derived HBM bytes per launch")
    ap.add_argument("--jit-wait-max-s", type=float, default=1500.0,
                    help="longest wait for background-compiled specialized kernels after warm-up")
    ap.add_argument("--micro", action="store_true", help="per-kernel bandwidth sweep")
    args = ap.parse_args(argv)
    wl = WORKLOADS[args.workload]
    args.qubits = wl["qubits"] if args.qubits is None else args.qubits
    args.layers = wl["layers"] if args.layers is None else args.layers
    if args.seed is None:
        args.seed = wl["seed"]
    return args


# BASELINE.json configs with a GPU workload of their own (SURVEY.md §8 d); C1 is the CPU GHZ
# plumbing check and C3 the f64 VQSE example (bench line's vqse_c3 block)
WORKLOADS = {
    "c2": {"qubits": 28, "layers": 20, "seed": 24, "config": "configs[1]",
           "name": "C2 layered random circuit (configs[1] generator: per layer a Haar q1 var gate "
                   "on every qubit + Haar q2 var brickwork, DiffQ1Density on every qubit)"},
    "c4": {"qubits": 30, "layers": 40, "seed": 30, "config": "configs[3]",
           "name": "C4 brickwall (configs[3]: 40 layers of Haar q2 var gates on (i, i+1), even then "
                   "odd, DiffQ1Density on every qubit)"},
    "c5": {"qubits": 33, "layers": 10000, "seed": 33, "config": "configs[4]",
           "name": "C5 deep random circuit (configs[4]: 10 000 gates, 50 % Haar q1, 35 % Haar q2, "
                   "15 % diagonal, DiffQ1Density on {0, n/2, n-2, n-1})"},
}


def workload_circuit(workload, n, layers, seed):
    """(instructions, var_gates) of a BASELINE workload (quantum_differentiable_circuit.workloads)."""
    from quantum_differentiable_circuit import workloads as W
    if workload == "c4":
        return W.brickwall_circuit(n, layers, seed)
    if workload == "c5":
        return W.deep_random_circuit(n, layers, seed)
    return W.layered_circuit(n, layers, seed)


def build_circuit(q, n, layers, seed, precision, comm=None, local_shards=None, devices=None,
                  workload="c2"):
    ins, var = workload_circuit(workload, n, layers, seed)
    c = q.circuit_class(precision)(n, comm=comm, local_shards=local_shards, devices=devices)
    for kind, pos in ins:
        c._push(kind, *pos)
    dt = c.dtype
    vg = [np.ascontiguousarray(g, dtype=dt) for g in var]
    return c, ins, vg


def sigma_z_cotangents(ndens, dt):
    # d/d rho of Re tr(rho sigma_z) is sigma_z^T; the qdc wiring conjugates it (circuit.py:193)
    return [np.ascontiguousarray(np.diag([1.0, -1.0]).astype(dt)) for _ in range(ndens)]


def dist_setup(args):
    """One process per GPU under any launcher that exports WORLD_SIZE / RANK / LOCAL_RANK
    (torch.distributed.run here, as the driver launches it): the ranks coordinate only through
    the circuit's own RCCL communicator (quantum_differentiable_circuit.distributed), so no
    second collective stack (torch's bundled RCCL, gloo) is loaded into the process."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def barrier(comm):
    if comm is not None and comm.world > 1:
        comm.barrier()


def max_over_ranks(x, comm):
    return comm.max(x) if comm is not None and comm.world > 1 else x


def select_device(local):
    # HIP device selection for the native library (it uses the current device)
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    err = hip.hipSetDevice(ctypes.c_int(local))
    if err != 0:
        raise RuntimeError(f"hipSetDevice({local}) failed: {err}")


def _cref_op_costs(ops, n, q1_pos, q2_pairs, dens1_pos, dens2_pairs, diag_pairs=()):
    """Seconds per gate kind of the reference algorithm (src/circuit.rs:164-429 over
    src/primitives.cu's kernels, restated in oracle/cpu_ref.c) on 2^n-amplitude host states:
    a gate forward (1 apply) + backward (uncompute, gradient reduction, pull-back); a density
    forward (1 reduction) + backward (conj_and_double into a new state, transposed apply, add).
    Means over the sampled positions."""
    from quantum_differentiable_circuit import workloads as W
    dt = ops.state_dtype
    rng = np.random.default_rng(0)
    f = np.empty(1 << n, dt)
    f.real = rng.standard_normal(1 << n)
    f.imag = rng.standard_normal(1 << n)
    b = f[::-1].copy()
    u2 = W.haar_unitary(rng, 2).astype(dt).reshape(-1)
    u4 = W.haar_unitary(rng, 4).astype(dt).reshape(-1)
    d4 = np.exp(1j * rng.standard_normal(4)).astype(dt)
    u2h, u2t = np.conj(u2.reshape(2, 2).T).reshape(-1), u2.reshape(2, 2).T.reshape(-1).copy()
    u4h, u4t = np.conj(u4.reshape(4, 4).T).reshape(-1), u4.reshape(4, 4).T.reshape(-1).copy()

    def timed(fn):
        t0 = time.perf_counter()
        fn()
        return time.perf_counter() - t0

    out = {}

    def q1(p):
        ops.apply_q1_gate(f, u2, p)
        ops.apply_q1_gate(f, u2h, p)
        ops.get_q1_grad(f, b, p)
        ops.apply_q1_gate(b, u2t, p)

    def q2(pr):
        ops.apply_q2_gate(f, u4, *pr)
        ops.apply_q2_gate(f, u4h, *pr)
        ops.get_q2_grad(f, b, *pr)
        ops.apply_q2_gate(b, u4t, *pr)

    def diag(pr):
        ops.apply_q2_gate_diag(f, d4, *pr)
        ops.apply_q2_gate_diag(f, np.conj(d4), *pr)
        ops.get_q2_grad_diag(f, b, *pr)
        ops.apply_q2_gate_diag(b, d4, *pr)

    def dens1(p):
        ops.get_q1_density(f, p)
        add = ops.conj_and_double(f)
        ops.apply_q1_gate(add, u2t, p)
        ops.add(add, b)

    def dens2(pr):
        ops.get_q2_density(f, *pr)
        add = ops.conj_and_double(f)
        ops.apply_q2_gate(add, u4t, *pr)
        ops.add(add, b)

    # untimed: OpenMP team start-up and first touch of every page by the team
    ops.copy(f)
    ops.apply_q1_gate(f, u2, 0)
    ops.apply_q1_gate(b, u2, 0)
    for key, fn, items in (("q1", q1, q1_pos), ("q2", q2, q2_pairs), ("diag", diag, diag_pairs),
                           ("dens1", dens1, dens1_pos), ("dens2", dens2, dens2_pairs)):
        if items:
            out[key] = float(np.mean([timed(lambda x=x: fn(x)) for x in items]))
    return out


def _cref_whole_call(ops, n, circuit, dt, psi0=None, cot=None):
    """Wall time of one forward + backward call of the reference algorithm
    (oracle.OracleCircuit: circuit.rs:164-429 driving the C kernels) on a whole circuit."""
    from oracle import oracle as O
    ins, var = circuit
    o = O.OracleCircuit(n, dt, ops=ops)
    for kind, pos in ins:
        o.add(kind, *pos)
    if psi0 is not None:
        o.set_state_from_vector(psi0)
    vg = [np.ascontiguousarray(g, dtype=ops.state_dtype) for g in var]
    t0 = time.perf_counter()
    dens = o.forward([], vg)
    cots = [np.ascontiguousarray(cot if cot is not None else np.diag([1.0, -1.0]), dtype=dt)
            for _ in dens]
    o.backward(cots, [], vg)
    return {"s": time.perf_counter() - t0, "ins": ins}


def cpu_baseline(args, n):
    """The reference's algorithm on the host cores (oracle/cpu_ref.c: its CUDA kernels' index
    rules in C/OpenMP, driven in circuit.rs's order by oracle.OracleCircuit: unfused, one kernel
    per step, uncompute + gradient + pull-back per gate backward, a new state per density
    injection), timed end to end on whole calls:
      value (c2): one whole forward + backward call of the GPU line's own step — the C2
        generator at full n with --cpu-layers layers (default: the step's 20) and all of C2's
        densities — at all threads;
      two_layer_call: a measured whole 2-layer call (density-heavy: its 28 densities are the
        same as the step's), a cross-check;
      projection: the per-kind fwd+bwd costs (q1 / q2 / density + injection) timed at sampled
        positions and projected onto the step's gate mix;
      single_thread: the per-kind projection at one thread (a whole call would take an hour);
      c3_vqse: one whole C3 loss-and-gradient call (n = 26 f64) when its projection is short.
    c4 / c5: the per-kind projection of the workload's gate mix at min(n, 30) qubits (a whole
    C5 call at n = 33 is hours of CPU time and three 64 GiB host states)."""
    # idle OpenMP threads sleep instead of spinning: spinning teams were starved on shared
    # hosts (64-100 ms for a 2 ms kernel in this container); read when libgomp loads
    os.environ.setdefault("OMP_WAIT_POLICY", "passive")
    from oracle.cref import CRefOps
    from quantum_differentiable_circuit import workloads as W
    dt = np.complex64 if args.precision == "f32" else np.complex128
    ins, _ = workload_circuit(args.workload, n, args.layers, args.seed)
    n_q1 = sum(1 for k, _ in ins if k == W.VAR_Q1)
    n_q2 = sum(1 for k, _ in ins if k == W.VAR_Q2)
    n_dg = sum(1 for k, _ in ins if k == W.VAR_Q2_DIAG)
    n_d1 = sum(1 for k, _ in ins if k == W.DIFF_Q1_DENSITY)
    ngates = n_q1 + n_q2 + n_dg
    res = {}
    t_all = time.perf_counter()
    ops = CRefOps(args.precision)
    threads = ops.threads()
    if args.workload != "c2":
        nc = min(n, args.cpu_qubits or 30)
        spread = [0, nc // 2, nc - 1]
        pairs = [(1, 0), (nc // 2 + 1, nc // 2), (nc - 1, nc - 2)]
        c = _cref_op_costs(ops, nc, spread, pairs, [0, nc - 1], [], pairs if n_dg else ())
        step = n_q1 * c["q1"] + n_q2 * c["q2"] + n_dg * c.get("diag", 0.0) + n_d1 * c["dens1"]
        scale = 2.0 ** (n - nc)  # HBM-bound kernels: time per gate ~ state size
        wall = time.perf_counter() - t_all
        return {"value": round(ngates / (step * scale), 6), "unit": "gate-applications/s (fwd+bwd)",
                "cores": threads, "kind": "port", "s_per_step": round(step * scale, 1),
                "sample": (f"per-kind projection: the reference's fwd+bwd cost per gate kind "
                           f"(oracle/cpu_ref.c kernels in circuit.rs order, OpenMP on {threads} "
                           f"threads) timed at n={nc} on sampled positions, projected onto the "
                           f"{args.workload} step's gate mix ({n_q1} q1, {n_q2} q2, {n_dg} diag, "
                           f"{n_d1} densities) and scaled by 2^({n}-{nc}) to n={n}; "
                           f"{wall:.0f} s of CPU time"),
                "per_gate_s_at_n": {k: round(v, 4) for k, v in c.items()}, "n_timed": nc}
    # whole calls, measured (one untimed layer first: OpenMP team start-up, page first touch)
    _cref_whole_call(ops, n, W.layered_circuit(n, 1, args.seed), dt)
    lay = args.cpu_layers or args.layers
    m2 = _cref_whole_call(ops, n, W.layered_circuit(n, 2, args.seed), dt)
    g2 = sum(1 for k, _ in m2["ins"] if k in (W.VAR_Q1, W.VAR_Q2))
    res["two_layer_call"] = {"s": round(m2["s"], 2), "gates": g2,
                             "value": round(g2 / m2["s"], 4)}
    mL = m2 if lay == 2 else _cref_whole_call(ops, n, W.layered_circuit(n, lay, args.seed), dt)
    gL = sum(1 for k, _ in mL["ins"] if k in (W.VAR_Q1, W.VAR_Q2))
    # the per-kind projection (earlier rounds' headline), as a cross-check
    spread = [0, n // 2, n - 1]
    c2 = _cref_op_costs(ops, n, spread, [(p + 1, p) for p in spread[:-1]] + [(n - 1, n - 2)],
                        [0, n - 1], [])
    step = n_q1 * c2["q1"] + n_q2 * c2["q2"] + n_d1 * c2["dens1"]
    res["projection"] = {"s_per_step": round(step, 2), "value": round(ngates / step, 4),
                         "per_gate_s": {k: round(v, 4) for k, v in c2.items()}}
    if lay == args.layers:
        res["projection"]["error_vs_measured_step"] = round((step - mL["s"]) / mL["s"], 4)
    ops.set_threads(1)
    c2s = _cref_op_costs(ops, n, [n // 2], [(n // 2 + 1, n // 2)], [n // 2], [])
    ops.set_threads(threads)
    step1 = n_q1 * c2s["q1"] + n_q2 * c2s["q2"] + n_d1 * c2s["dens1"]
    res["single_thread"] = {"value": round(ngates / step1, 4), "cores": 1,
                            "s_per_step": round(step1, 2), "kind": "per-kind projection",
                            "per_gate_s": {k: round(v, 4) for k, v in c2s.items()}}
    # C3: the VQSE circuit at the example's size, f64
    n3, layers3 = 26, 26
    ops64 = CRefOps("f64")
    c3 = _cref_op_costs(ops64, n3, [0, n3 // 2, n3 - 1], [], [], [(0, 1), (12, 13), (0, n3 - 1)],
                        [(0, 1), (12, 13), (0, n3 - 1)])
    call = layers3 * n3 * (c3["diag"] + c3["q1"]) + n3 * c3["dens2"]
    res["c3_vqse"] = {"projected_s_per_call": round(call, 2), "qubits": n3, "layers": layers3,
                      "dtype": "c128 (f64)", "cores": ops64.threads(),
                      "per_gate_s": {k: round(v, 4) for k, v in c3.items()}}
    if call <= args.cpu_c3_max_s:
        try:
            p = np.random.default_rng(42).normal(size=2 * layers3)
            ins3 = W.vqse_ising(n3, layers3)
            gates3 = W.vqse_gates(p, n3)
            psi3 = np.full(1 << n3, 1.0 / np.sqrt(1 << n3), np.complex128)
            m3 = _cref_whole_call(ops64, n3, (ins3, gates3), np.complex128, psi0=psi3,
                                  cot=W.tfim_term(1.0).T.conj())
            res["c3_vqse"].update({"s_per_loss_grad_call": round(m3["s"], 2),
                                   "projection_error": round((call - m3["s"]) / m3["s"], 4)})
        except Exception as e:  # noqa: BLE001
            res["c3_vqse"]["measured_error"] = f"{type(e).__name__}: {e}"[:300]
    else:
        res["c3_vqse"]["s_per_loss_grad_call"] = f"not measured: projected {call:.0f} s > --cpu-c3-max-s"
    wall = time.perf_counter() - t_all
    whole = lay == args.layers
    return {"value": round(gL / mL["s"], 4), "unit": "gate-applications/s (fwd+bwd)",
            "cores": threads, "kind": "port", "s_per_call": round(mL["s"], 2),
            "sample": (f"measured: one whole forward + backward call of the C2 generator at full "
                       f"n={n} {args.precision} with {lay} layers ({gL} gates) and its {n_d1} "
                       f"densities" + (" - the GPU line's own step" if whole else "") +
                       f", the reference's algorithm (oracle/cpu_ref.c kernels in circuit.rs "
                       f"order: unfused, per-gate uncompute + gradient + pull-back, a new state "
                       f"per density injection), OpenMP on {threads} threads, timed end to end; "
                       f"two_layer_call / projection / single_thread: cross-checks; c3_vqse: one "
                       f"whole n=26 f64 VQSE call; {wall:.0f} s of CPU time"),
            **res}


def gate_kernel_sweep(args, n, verbose=False):
    """Single-gate kernels (fusion off): the north star's >= 70 % HBM target on 1- and 2-qubit
    gate application at n=28 f32, over the SURVEY §8(d) sweep: q1 at every position 0..n-1 and
    q2 (dense and diagonal) at the pairs (0,1), (1,0), (5,20), (26,27), (27,0), (1,2), (3,9),
    (14,13); per cell the median over 20 fwd+bwd iterations (after 3 warm-ups) of each
    kernel's per-launch HIP-event time (apply, reverse = uncompute + gradient + pull-back,
    inject, density).  Returns every cell and the minimum one."""
    rows = micro(args, n, verbose=verbose)
    for lab, k, _, ms, gbs in rows:  # every cell on stderr (the JSON line keeps the summary)
        print(f"[micro] {lab:10s} {k:18s} {ms:8.4f} ms {gbs:8.1f} GB/s {gbs / HBM_PEAK_GBS:6.1%}",
              file=sys.stderr, flush=True)
    cells = [{"case": lab, "kernel": k, "ms": round(ms, 4), "GB/s": round(gbs, 1),
              "frac": round(gbs / HBM_PEAK_GBS, 4)} for lab, k, _, ms, gbs in rows]
    # the target's cells: gate application and the reverse sweep's per-gate kernel (not the
    # reductions or the density injection, which are reported beside them)
    gate = [c for c in cells if c["kernel"].startswith(("apply_", "reverse_"))]
    worst = min(gate, key=lambda c: c["frac"]) if gate else None
    per = {}
    for c in cells:
        lo, hi = per.get(c["kernel"], (1e9, 0.0))
        per[c["kernel"]] = (min(lo, c["frac"]), max(hi, c["frac"]))
    return {"micro_min": worst,
            "cells": len(gate), "cells_below_70pct": [f"{c['kernel']} {c['case']} {c['frac']:.3f}"
                                                       for c in gate if c["frac"] < 0.70],
            "frac_range_by_kernel": {k: [round(lo, 4), round(hi, 4)] for k, (lo, hi) in sorted(per.items())},
            "method": "median of 20 fwd+bwd iterations after 3 warm-ups, HIP events per launch, "
                      "fusion off, a fresh circuit per case, n=%d %s" % (n, args.precision)}


def dense_gate_sample(args, n):
    """Dense k-qubit gates (k = 3, 4, 5; include/qdc/dense.h) on the matrix cores at n: 8
    random unitaries per k at mixed positions, per-kernel HIP-event time on the primitives'
    stream, algorithmic bytes 2S and FLOPs 8 * 2^k per amplitude."""
    import quantum_differentiable_circuit as q
    dt = np.complex64 if args.precision == "f32" else np.complex128
    rng = np.random.default_rng(2)
    t = q.QuantizedTensor.new_standard(n, precision=args.precision)
    mats = {k: [np.ascontiguousarray(O_haar(rng, 1 << k), dtype=dt) for _ in range(8)]
            for k in (3, 4, 5)}
    poss = {k: [list(rng.permutation(n)[:k]) for _ in range(8)] for k in (3, 4, 5)}
    for k in (3, 4, 5):  # warm-up
        t.apply_qk_gate(mats[k][0], poss[k][0])
    q.primitives_sync(args.precision)
    q.primitives_profile(True, args.precision)
    for k in (3, 4, 5):
        for u, pos in zip(mats[k], poss[k]):
            t.apply_qk_gate(u, pos)
    stats = q.primitives_profile_collect(args.precision)
    q.primitives_profile(False, args.precision)
    del t
    out = {}
    for k in (3, 4, 5):
        s = stats.get(f"qk{k}")
        if s and s["total_ms"] > 0:
            gbs = s["algo_bytes"] / (s["total_ms"] * 1e-3) / 1e9
            out[f"qk{k}"] = {"GB/s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                             "TFLOP/s": round(s["algo_flops"] / (s["total_ms"] * 1e-3) / 1e12, 2),
                             "launches": s["launches"],
                             "avg_ms": round(s["total_ms"] / s["launches"], 4)}
    return out


def vqse_sample(precision="f64", steps=3):
    """Config C3 (example_vqse_ising.py at its own size: n = 26, 26 layers, |+>^n) in either
    precision — BASELINE.json names f64, the example itself runs complex64
    (example_vqse_ising.py:58,87-89): wall seconds per loss-and-gradient call (the number
    example:133 prints), and the HBM roofline and VALU rate of the call's dominant kernel (HIP
    events on the circuit's stream)."""
    from qdc import AutoGradCircuit
    from quantum_differentiable_circuit import workloads as W
    n, layers = 26, 26
    ac = AutoGradCircuit(n, precision=precision)
    ac.set_state_from_vector(np.ones(1 << n, dtype=ac.dtype) / np.sqrt(1 << n))
    for kind, pos in W.vqse_ising(n, layers):
        if kind == W.VAR_Q2_DIAG:
            ac.add_q2_var_gate_diag(*pos)
        elif kind == W.VAR_Q1:
            ac.add_q1_var_gate(*pos)
        else:
            ac.get_q2_dens_op_with_grad(*pos)
    _, fwd_circ = ac.build()

    def f(gates):
        return fwd_circ.vjp(gates, [])

    h = W.tfim_term(1.0)
    p = np.random.default_rng(42).normal(size=2 * layers)
    W.vqse_loss_and_grad(f, p, n, h)  # warm-up
    ac.circuit.profile(True)
    ac.circuit.host_times(reset=True)
    t0 = time.perf_counter()
    for _ in range(steps):
        e, _ = W.vqse_loss_and_grad(f, p, n, h)
    dt = (time.perf_counter() - t0) / steps
    stats = ac.circuit.profile_collect()
    ac.circuit.profile(False)
    out = {"s_per_loss_grad_call": round(dt, 4), "energy": round(e, 6), "qubits": n,
           "layers": layers, "gates": 2 * n * layers,
           "dtype": "c128 (f64)" if precision == "f64" else "c64 (f32)", "calls": steps}
    dom_name, dom = max(stats.items(), key=lambda kv: kv[1]["total_ms"])
    avg = dom["total_ms"] / dom["launches"]
    gbs = dom["algo_bytes"] / dom["launches"] / (avg * 1e-3) / 1e9
    out["device_ms_per_call"] = round(sum(v["total_ms"] for v in stats.values()) / steps, 2)
    out["host_ms_per_call"] = {d: {k: round(v / steps, 3) for k, v in t.items() if k != "calls"}
                               for d, t in ac.circuit.host_times().items()}
    out["roofline"] = {"bound": "hbm", "kernel": dom_name, "achieved": round(gbs, 1),
                       "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                       "avg_launch_ms": round(avg, 4), "launches_per_call": dom["launches"] // steps,
                       "algo_bytes_per_launch": dom["algo_bytes"] / dom["launches"]}
    if dom.get("algo_flops"):
        tf = dom["algo_flops"] / dom["launches"] / (avg * 1e-3) / 1e12
        out["compute"] = {"bound": "valu", "kernel": dom_name, "achieved": round(tf, 2),
                          "peak": VALU_PEAK_TFLOPS[precision], "unit": "TFLOP/s",
                          "frac": round(tf / VALU_PEAK_TFLOPS[precision], 4)}
    out["kernels"] = {k: {"launches": v["launches"] // steps,
                          "avg_ms": round(v["total_ms"] / v["launches"], 4)}
                      for k, v in sorted(stats.items(), key=lambda kv: -kv[1]["total_ms"])}
    return out


def abi_unfused_sample(args, n):
    """The same C2 step through the 18-function C ABI in the reference's own call sequence
    (quantum_differentiable_circuit.abi_circuit.AbiCircuit, circuit.rs:164-429 over
    QuantizedTensor): what a Rust host linking libqdc per INTEGRATION.md §1 gets.  One step
    (forward + backward), wall time; every gradient is a host sync as in the reference."""
    from quantum_differentiable_circuit import workloads as W
    from quantum_differentiable_circuit.abi_circuit import AbiCircuit
    ins, var = W.layered_circuit(n, args.layers, args.seed)
    a = AbiCircuit(n, args.precision)
    for kind, pos in ins:
        a.add(kind, *pos)
    dt = a.dtype
    vg = [np.ascontiguousarray(g, dtype=dt) for g in var]
    warm = AbiCircuit(n, args.precision)  # every kernel variant once
    wins, wvar = W.layered_circuit(n, 1, args.seed)
    for kind, pos in wins:
        warm.add(kind, *pos)
    wd = warm.forward([], [np.ascontiguousarray(g, dtype=dt) for g in wvar])
    warm.backward(sigma_z_cotangents(len(wd), dt), [], [np.ascontiguousarray(g, dtype=dt) for g in wvar])
    del warm
    t0 = time.perf_counter()
    d = a.forward([], vg)
    g = a.backward(sigma_z_cotangents(len(d), dt), [], vg)
    a.state.get_cpu_state_copy() if n <= 20 else None
    from quantum_differentiable_circuit import primitives_sync
    primitives_sync(args.precision)
    el = time.perf_counter() - t0
    assert all(np.isfinite(x).all() for x in g)
    return {"value": round(len(vg) / el, 3), "unit": "gate-applications/s (fwd+bwd)",
            "s_per_step": round(el, 3), "gates": len(vg), "densities": len(d),
            "path": "AbiCircuit: circuit.rs over the 18 primitives (unfused, one kernel per step, "
                    "host sync per gradient, a new state per density injection)"}


def micro(args, n=None, verbose=True, q1_positions=None, q2_pairs=None):
    """Per-kernel bandwidth: each gate kind at every position, forward and fused reverse
    (single-gate kernels: fusion off).  Returns (case, kernel, launches, median ms, GB/s) rows."""
    import quantum_differentiable_circuit as q
    n = args.qubits if n is None else n
    prec = args.precision
    dt = np.complex64 if prec == "f32" else np.complex128
    rng = np.random.default_rng(0)
    rows = []

    def run(label, setup):
        """the median over 20 fwd+bwd iterations (after 3 warm-ups) of each
        kernel's per-launch HIP-event time in the iteration."""
        old = os.environ.get("QDC_FUSE")
        os.environ["QDC_FUSE"] = "0"
        try:
            c = q.circuit_class(prec)(n)
        finally:
            if old is None:
                os.environ.pop("QDC_FUSE", None)
            else:
                os.environ["QDC_FUSE"] = old
        var = setup(c)
        cots = sigma_z_cotangents(1, dt)
        for _ in range(3):
            c.forward([], var)
            c.backward(cots, [], var)
        per = {}
        for _ in range(20):
            c.profile(True)
            c.forward([], var)
            c.backward(cots, [], var)
            for k, s in c.profile_collect().items():
                if s["total_ms"] > 0 and k not in ("finalize",):
                    per.setdefault(k, []).append((s["total_ms"] / s["launches"], s["algo_bytes"] / s["launches"],
                                                  s["launches"]))
        c.profile(False)
        for k, v in per.items():
            ms = float(np.median([x[0] for x in v]))
            gbs = v[0][1] / (ms * 1e-3) / 1e9
            rows.append((label, k, v[0][2], ms, gbs))
            if verbose:
                print(f"{label:14s} {k:18s} n={v[0][2]:4d} {ms:8.3f} ms {gbs:8.1f} GB/s  "
                      f"{gbs / HBM_PEAK_GBS:6.1%}  (median of {len(v)})", flush=True)
        del c

    reps = 8
    for pos in (range(n) if q1_positions is None else q1_positions):
        def s1(c, pos=pos):
            for _ in range(reps):
                c.add_q1_var_gate(pos)
            c.get_q1_dens_op_with_grad(pos)
            return [np.ascontiguousarray(O_haar(rng, 2), dtype=dt) for _ in range(reps)]
        run(f"q1 {pos}", s1)
    pairs = [(0, 1), (1, 0), (5, 20), (26, 27), (27, 0), (1, 2), (3, 9), (14, 13)]
    for pos2, pos1 in (pairs if q2_pairs is None else q2_pairs):
        if max(pos2, pos1) >= n:
            continue

        def s2(c, pos2=pos2, pos1=pos1):
            for _ in range(reps):
                c.add_q2_var_gate(pos2, pos1)
            for _ in range(reps):
                c.add_q2_var_gate_diag(pos2, pos1)
            c.get_q1_dens_op_with_grad(pos1)
            return ([np.ascontiguousarray(O_haar(rng, 4), dtype=dt) for _ in range(reps)]
                    + [np.exp(1j * rng.standard_normal(4)).astype(dt) for _ in range(reps)])
        run(f"q2 {pos2},{pos1}", s2)
    return rows


def O_haar(rng, k):
    from quantum_differentiable_circuit import workloads as W
    return W.haar_unitary(rng, k)


def main():
    args = parse()
    world, rank, local = dist_setup(args)
    select_device(local)
    import quantum_differentiable_circuit as q
    if args.micro:
        micro(args)
        return

    n = args.qubits
    comm = devices = None
    if world > 1:  # one process per GPU (torchrun): RCCL id through a file, no torch in the product
        from quantum_differentiable_circuit.distributed import Communicator
        comm = Communicator(args.precision, rank=rank, world=world, device=local)
    elif args.gpus > 1:  # one plain process driving every GPU (ncclCommInitAll)
        devices = list(range(args.gpus))
    elif args.local_streams and args.local_streams > 1:  # the same plumbing, one GPU
        devices = [0] * args.local_streams
    c, ins, vg = build_circuit(q, n, args.layers, args.seed, args.precision, comm,
                               args.local_shards, devices, args.workload)
    ngates = len(vg)
    cots = sigma_z_cotangents(sum(1 for k, _ in ins if k in (12, 13)), c.dtype)
    wl = WORKLOADS[args.workload]
    remaps = 0
    shards = world if world > 1 else (len(devices) if devices else (args.local_shards or 1))
    if shards > 1:
        instr = [(k, *p) for k, p in ins]
        # the mirrored forward's plan; its backward undoes each of its remaps (qdc_circuit.hpp
        # unremap), unless QDC_MIRROR=0 (the backward plans its own)
        if os.environ.get("QDC_MIRROR", "1") != "0":
            f_ops, _ = q.plan(n, shards, instr, 3, precision=args.precision)
            remaps = 2 * sum(o["type"] == "remap" for o in f_ops)
        else:
            f_ops, end = q.plan(n, shards, instr, 1, precision=args.precision)
            b_ops, _ = q.plan(n, shards, instr, 2, start_phys=end, precision=args.precision)
            remaps = sum(o["type"] == "remap" for o in f_ops + b_ops)

    tw = time.perf_counter()
    with heartbeat("warm-up"):
        for _ in range(args.warmup):
            c.forward([], vg)
            c.backward(cots, [], vg)
        c.synchronize()
    # a program with more distinct specialized kernels than QDC_SPEC_MAX (C5's deep random
    # circuit) compiles them in the background while generic kernels run its passes: wait for
    # them (progress on stderr), then one more untimed step loads them
    # The decision is collective: the extra step issues RCCL all-to-alls and all-reduces, so every
    # rank runs it when any rank still has kernels queued, and the wait loop ends on the same
    # iteration everywhere (max over ranks of what is left and of the time waited).
    jit_bg_s = 0.0
    if max_over_ranks(float(q.jit_stats(args.precision)["queued"]), comm) > 0:
        tj = time.perf_counter()
        while True:
            left = q.jit_wait(30.0, args.precision)
            print(f"[bench] rank {rank}: {left} specialized kernels still compiling "
                  f"({time.perf_counter() - tj:.0f} s)", file=sys.stderr, flush=True)
            left_all = max_over_ranks(float(left), comm)
            waited = max_over_ranks(time.perf_counter() - tj, comm)
            if left_all == 0 or waited > args.jit_wait_max_s:
                break
        jit_bg_s = time.perf_counter() - tj
        with heartbeat("warm-up on the specialized passes"):
            c.forward([], vg)
            c.backward(cots, [], vg)
            c.synchronize()
    warmup_s = time.perf_counter() - tw  # includes the specialized kernels' compilation

    # QDC_BENCH_UNPROFILED_STEPS=K (experiment): K more timed steps without the per-launch HIP
    # events first, reported as unprofiled_ms_per_step (what the events cost the step)
    unprof = int(os.environ.get("QDC_BENCH_UNPROFILED_STEPS", "0"))
    unprof_ms = None
    if unprof > 0:
        barrier(comm)
        c.synchronize()
        tu = time.perf_counter()
        for _ in range(unprof):
            c.forward([], vg)
            c.backward(cots, [], vg)
        c.synchronize()
        unprof_ms = max_over_ranks(time.perf_counter() - tu, comm) / unprof * 1e3
    c.profile(True)
    c.host_times(reset=True)
    barrier(comm)
    c.synchronize()
    with heartbeat("timed steps"):
        t0 = time.perf_counter()
        for _ in range(args.steps):
            dens = c.forward([], vg)
            grads = c.backward(cots, [], vg)
        c.synchronize()
        elapsed = time.perf_counter() - t0
    barrier(comm)
    stats = c.profile_collect()
    c.profile(False)
    # host milliseconds per step by phase (rank 0): scheduling and program building sit before a
    # call's first launch, so they are device idle time unless the previous call still runs
    ht = c.host_times()
    host_ms = {d: {k: round(v / args.steps, 3) for k, v in ht[d].items() if k != "calls"}
               for d in ht}

    # per rank: the specialized-kernel cache (compile / wait seconds, kernels compiled by this
    # rank: one rank compiles each kernel of a job) and the all-to-all time per step, so a first
    # multi-GPU run separates JIT warm-up and exchange cost from the passes
    js = q.jit_stats(args.precision)
    a2a = stats.get("alltoall", {})
    mine = [js["total_s"], js["compile_s"], js["wait_s"], float(js["compiled"]),
            a2a.get("total_ms", 0.0) / args.steps, a2a.get("launches", 0) / args.steps, warmup_s,
            jit_bg_s, float(js["launched"])]
    nf = len(mine)
    per_rank_vals = [mine]
    if comm is not None and comm.world > 1:
        vec = [0.0] * (nf * world)
        vec[nf * rank:nf * rank + nf] = mine
        allv = comm.allreduce(vec)
        per_rank_vals = [allv[nf * r:nf * r + nf] for r in range(world)]
    per_rank = [{"rank": r, "jit_s": round(v[0], 3), "jit_compile_s": round(v[1], 3),
                 "jit_wait_s": round(v[2], 3), "kernels_compiled": int(v[3]),
                 "alltoall_ms_per_step": round(v[4], 3), "alltoalls_per_step": v[5],
                 "warmup_s": round(v[6], 2), "jit_background_wait_s": round(v[7], 2),
                 "specialized_launches": int(v[8])} for r, v in enumerate(per_rank_vals)]

    elapsed = max_over_ranks(elapsed, comm)
    value = ngates * args.steps / elapsed  # the one sharded circuit's gate applications

    # dominant HBM kernel = the one with the largest share of measured device time
    dom_name, dom = max(((k, v) for k, v in stats.items() if k != "alltoall"),
                        key=lambda kv: kv[1]["total_ms"])
    avg_ms = dom["total_ms"] / dom["launches"]
    bytes_per_launch = dom["algo_bytes"] / dom["launches"]
    dom_flops = dom.get("algo_flops", 0.0) / dom["launches"]
    valu_peak = VALU_PEAK_TFLOPS[args.precision]
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    # HBM bytes per launch from the PMC passes (FETCH_SIZE / WRITE_SIZE, tools/pmc_summary.py),
    # quoted only when they were collected on this very library build
    traffic, traffic_src = None, None
    pmc_path = Path(args.pmc) if args.pmc else ROOT / "profiles" / "pmc_traffic.json"
    if pmc_path.exists():
        try:
            import hashlib
            pmc = json.loads(pmc_path.read_text())
            lib = Path(__import__("quantum_differentiable_circuit._native", fromlist=["x"]).lib_path(
                args.precision))
            sha = hashlib.sha256(lib.read_bytes()).hexdigest()[:16]
            # the PMC passes run the default workload (C2 at n = 28): per-launch bytes of
            # another workload or size are not this line's
            if args.workload != "c2" or n != 28:
                traffic_src = f"{pmc_path.name} measures the C2 n=28 step, not this workload"
            elif args.precision == "f32" and pmc.get("lib_sha16") == sha:
                traffic, traffic_src = pmc.get(dom_name), f"{pmc_path.name} (build {sha})"
            else:
                traffic_src = f"{pmc_path.name} is from another build ({pmc.get('lib_sha16')} != {sha})"
        except Exception as e:  # noqa: BLE001
            traffic_src = f"unreadable: {e}"[:200]
    kernels = {k: {"launches": v["launches"], "avg_ms": round(v["total_ms"] / v["launches"], 4),
                   "GB/s": round(v["algo_bytes"] / (v["total_ms"] * 1e-3) / 1e9, 1)
                   if v["total_ms"] > 0 else None,
                   "TFLOP/s": round(v["algo_flops"] / (v["total_ms"] * 1e-3) / 1e12, 2)
                   if v["total_ms"] > 0 and v.get("algo_flops") else None,
                   "share": round(v["total_ms"] / sum(s["total_ms"] for s in stats.values()), 4)}
               for k, v in sorted(stats.items(), key=lambda kv: -kv[1]["total_ms"])}

    # sanity: the loss gradient is finite and the densities are traces of 1
    # (QDC_BENCH_ABLATION: timing-only builds that skip part of the kernel work)
    if not os.environ.get("QDC_BENCH_ABLATION"):
        assert all(np.isfinite(g).all() for g in grads)
        assert all(abs(np.trace(d) - 1) < 1e-3 for d in dens)

    # the fused path against the per-gate roofline: every gate costs 2S forward and 4S in the
    # reverse sweep (SURVEY.md §8 d) if applied one HBM pass at a time
    state_bytes = (1 << n) * (8 if args.precision == "f32" else 16)
    ngpu = world if world > 1 else (len(set(devices)) if devices else 1)
    eff = ngates * 6 * state_bytes / (elapsed / args.steps) / 1e9 / ngpu
    effective = {"per_gpu_GB/s": round(eff, 1), "x_hbm_peak": round(eff / HBM_PEAK_GBS, 3),
                 "definition": "gates x (2S fwd + 4S bwd) per step / step time, per GPU"}
    # the all-to-all of sharded runs: bytes each shard sends to the others per all-to-all over
    # the exchange's event time, per GPU, against the link it crosses (one GPU per process or
    # per shard: xGMI; a one-GPU rehearsal: device copies through HBM)
    exchange = None
    a2a = stats.get("alltoall")
    if shards > 1 and a2a and a2a["launches"] > 0 and a2a["total_ms"] > 0:
        per_gpu = shards // ngpu  # shards a GPU holds (every shard's events span its GPU's copies)
        avg = a2a["total_ms"] / a2a["launches"]
        sent = a2a["algo_bytes"] / a2a["launches"] * per_gpu  # bytes per GPU per all-to-all
        gbs = sent / (avg * 1e-3) / 1e9
        if ngpu > 1:
            link, peak = (f"xGMI, {ngpu - 1} of the 7 point-to-point links per GPU at "
                          f"{XGMI_LINK_GBS:.0f} GB/s each"), (ngpu - 1) * XGMI_LINK_GBS
        else:
            link, peak = ("rehearsal: device copies on one GPU (each byte read and written in "
                          "HBM)"), HBM_PEAK_GBS / 2
        nrec = 1 if world > 1 else shards  # event records per all-to-all (one per local shard)
        exchange = {"alltoalls_per_step": round(a2a["launches"] / args.steps / nrec, 2),
                    "avg_ms": round(avg, 4), "bytes_per_gpu": sent,
                    "alltoall_GB/s": round(gbs, 1), "link": link, "link_peak_GB/s": peak,
                    "frac": round(gbs / peak, 4),
                    "ms_per_step": round(a2a["total_ms"] / args.steps / nrec, 3)}

    gate_kernels = dense_kernels = vqse = vqse32 = abi = None
    # (the auxiliary samples and the CPU baseline belong to the one-GPU headline: a sharded run —
    # any number of processes, GPUs or local shards — reports its own step and exchange only)
    if rank == 0 and shards == 1 and not args.no_gate_sample and args.workload == "c2":
        # auxiliary samples: a failure there is reported in the line, never loses the headline
        def aux(fn, *a):
            try:
                return fn(*a)
            except Exception as e:  # noqa: BLE001
                return {"error": f"{type(e).__name__}: {e}"[:300]}
        with heartbeat("auxiliary samples"):
            gate_kernels = aux(gate_kernel_sweep, args, n)
            dense_kernels = aux(dense_gate_sample, args, n)
            vqse = aux(vqse_sample, "f64")
            vqse32 = aux(vqse_sample, "f32")
            abi = aux(abi_unfused_sample, args, n)

    cpu = None
    if rank == 0 and shards == 1 and not args.no_cpu_baseline:
        try:
            with heartbeat("CPU baseline (the reference's algorithm on the host cores)"):
                cpu = cpu_baseline(args, args.cpu_qubits or n)
        except Exception as e:  # noqa: BLE001
            cpu = {"error": f"{type(e).__name__}: {e}"[:300]}

    if rank == 0:
        state_gib = (1 << n) * (8 if args.precision == "f32" else 16) / 2**30
        line = {
            "metric": "gate-applications/sec (fwd+bwd) at n qubits",
            "value": round(value, 3),
            "unit": "gate-applications/s",
            "n_gpus": ngpu,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "c64 (f32)" if args.precision == "f32" else "c128 (f64)",
            "data": "synthetic (seeded Haar-random gates, |0..0> initial state)",
            "config": {"workload": f"{wl['name']} at n={n}, fwd+bwd",
                       "baseline_config": f"BASELINE.json {wl['config']}", "bench_workload": args.workload,
                       "qubits": n, ("gates" if args.workload == "c5" else "layers"): args.layers,
                       "gates_per_step": ngates, "seed": args.seed,
                       "densities_per_step": len(cots), "state_GiB": state_gib,
                       "parallelism": (f"state sharded over {world} GPUs by high qubits, "
                                       f"RCCL all-to-all remaps, one process per GPU") if world > 1 else
                                      (f"state sharded over {ngpu} GPUs by high qubits, RCCL "
                                       f"all-to-all remaps, one process (ncclCommInitAll)")
                                      if devices and ngpu > 1 else
                                      (f"rehearsal: {len(devices)} shards on one GPU, one stream "
                                       f"each (event-ordered device copies)")
                                      if devices else
                                      (f"rehearsal: {shards} shards on one GPU (device copies)"
                                       if shards > 1 else "single GPU"),
                       "remaps_per_step": remaps},
            "roofline": {"bound": "hbm", "kernel": dom_name, "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "algo_bytes_per_launch": bytes_per_launch,
                         "avg_launch_ms": round(avg_ms, 4)},
            # fused passes are VALU-bound: their FLOP rate against the vector peak
            "compute": ({"bound": "valu", "kernel": dom_name,
                         "achieved": round(dom_flops / (avg_ms * 1e-3) / 1e12, 2),
                         "peak": valu_peak, "unit": "TFLOP/s",
                         "frac": round(dom_flops / (avg_ms * 1e-3) / 1e12 / valu_peak, 4),
                         "algo_flops_per_launch": dom_flops}
                        if dom_flops > 0 else None),
            "kernels": kernels,
            "host_ms_per_step": host_ms,
            "ranks": per_rank,
            "effective_gate_bandwidth": effective,
            "micro_min": (gate_kernels or {}).get("micro_min") if isinstance(gate_kernels, dict) else None,
            "gate_kernels": gate_kernels,
            "dense_gate_kernels": dense_kernels,
            "vqse_c3": vqse,
            "vqse_c3_f32": vqse32,
            "exchange": exchange,
            "unprofiled_ms_per_step": round(unprof_ms, 3) if unprof_ms else None,
            "abi_unfused": abi,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()

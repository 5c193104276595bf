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

Multi-GPU (python -m torch.distributed.run ... bench.py --gpus N): strong scaling — the SAME
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--qubits", type=int, default=28)
    ap.add_argument("--layers", type=int, default=20)
    ap.add_argument("--precision", default="f32", choices=["f32", "f64"])
    ap.add_argument("--seed", type=int, default=24)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--local-shards", type=int, default=None,
                    help="rehearse the sharded data path on one GPU (G shards, device copies in "
                         "place of the RCCL all-to-all); not a multi-GPU measurement")
    ap.add_argument("--no-gate-sample", action="store_true",
                    help="skip the single-gate (fusion off) kernel sample")
    ap.add_argument("--cpu-gates", type=int, default=12,
                    help="gates of the CPU baseline sample (the workload's first gates, full n)")
    ap.add_argument("--cpu-densities", type=int, default=4)
    ap.add_argument("--cpu-qubits", type=int, default=None)
    ap.add_argument("--pmc", default=None, help="JSON with PMC-derived HBM bytes per launch")
    ap.add_argument("--micro", action="store_true", help="per-kernel bandwidth sweep")
    return ap.parse_args()


def build_circuit(q, n, layers, seed, precision, comm=None, local_shards=None):
    from quantum_differentiable_circuit import workloads as W  # synthetic C2 workload
    ins, var = W.layered_circuit(n, layers, seed)
    c = q.circuit_class(precision)(n, comm=comm, local_shards=local_shards)
    for kind, pos in ins:
        c._push(kind, *pos)
    dt = c.dtype
    vg = [np.ascontiguousarray(g, dtype=dt) for g in var]
    return c, ins, vg


def sigma_z_cotangents(ndens, dt):
    # d/d rho of Re tr(rho sigma_z) is sigma_z^T; the qdc wiring conjugates it (circuit.py:193)
    return [np.ascontiguousarray(np.diag([1.0, -1.0]).astype(dt)) for _ in range(ndens)]


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x, world):
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x, world):
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def select_device(local):
    # HIP device selection for the native library (it uses the current device)
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    err = hip.hipSetDevice(ctypes.c_int(local))
    if err != 0:
        raise RuntimeError(f"hipSetDevice({local}) failed: {err}")


def cpu_baseline(args, n):
    """Time the oracle's C/OpenMP restatement of the reference algorithm (unfused uncompute /
    grad / pull-back and allocate-conj-gate-add density injection, circuit.rs:266-429) on a
    bounded sample of the same workload: its first `cpu_gates` gates and `cpu_densities`
    DiffQ1Density outputs, at full n."""
    from oracle import oracle as O
    from oracle.cref import CRefOps
    ops = CRefOps(args.precision)
    ins, var = O.layered_circuit(n, args.layers, args.seed)
    gates = [(k, p) for k, p in ins if k < 10][:args.cpu_gates]
    dens_ins = [(k, p) for k, p in ins if k >= 10][:args.cpu_densities]
    dt = ops.state_dtype
    o = O.OracleCircuit(n, dt, ops=ops)
    for kind, pos in gates + dens_ins:
        o.add(kind, *pos)
    var = var[:len(gates)]
    t0 = time.perf_counter()
    dens = o.forward([], var)
    o.backward(sigma_z_cotangents(len(dens), dt), [], var)
    dt_s = time.perf_counter() - t0
    return {"value": len(gates) / dt_s, "unit": "gate-applications/s (fwd+bwd)",
            "cores": ops.threads(), "kind": "port",
            "sample": f"first {len(gates)} gates + {len(dens)} DiffQ1Density of the same "
                      f"circuit at n={n} {args.precision}, fwd+bwd in {dt_s:.1f} s "
                      f"(oracle/cpu_ref.c, OpenMP, reference algorithm unfused)"}


def gate_kernel_sample(args, n):
    """Single-gate kernels (fusion off): the north star's >= 70 % HBM target is on 1- and
    2-qubit gate application at n=28 f32.  One circuit with q1 / q2 gates at low, middle and
    high positions (every kernel family), fwd+bwd x3, per-kernel algorithmic GB/s."""
    import quantum_differentiable_circuit as q
    dt = np.complex64 if args.precision == "f32" else np.complex128
    rng = np.random.default_rng(1)
    os.environ["QDC_FUSE"] = "0"
    try:
        c = q.circuit_class(args.precision)(n)
    finally:
        os.environ.pop("QDC_FUSE", None)
    var = []
    for _ in range(2):
        for pos in (0, 1, n // 2, n - 1):
            c.add_q1_var_gate(pos)
            var.append(np.ascontiguousarray(O_haar(rng, 2), dtype=dt))
        for pos2, pos1 in ((1, 0), (n - 1, 0), (n // 2 + 1, n // 2), (n - 1, n - 2)):
            c.add_q2_var_gate(pos2, pos1)
            var.append(np.ascontiguousarray(O_haar(rng, 4), dtype=dt))
    c.get_q1_dens_op_with_grad(0)
    cot = sigma_z_cotangents(1, dt)
    c.forward([], var)
    c.backward(cot, [], var)
    c.profile(True)
    for _ in range(3):
        c.forward([], var)
        c.backward(cot, [], var)
    stats = c.profile_collect()
    c.profile(False)
    del c
    out = {}
    for k in ("apply_q1", "apply_q2", "reverse_q1", "reverse_q2"):
        if k in stats and stats[k]["total_ms"] > 0:
            gbs = stats[k]["algo_bytes"] / (stats[k]["total_ms"] * 1e-3) / 1e9
            out[k] = {"GB/s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                      "launches": stats[k]["launches"],
                      "avg_ms": round(stats[k]["total_ms"] / stats[k]["launches"], 4)}
    return out


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


def vqse_sample(steps=3):
    """Config C3 (example_vqse_ising.py at its own size: n = 26, 26 layers, f64, |+>^n): wall
    seconds per loss-and-gradient call, the number the example prints (example:133)."""
    sys.path.insert(0, str(ROOT / "examples"))
    import vqse_ising
    from quantum_differentiable_circuit import workloads as W
    n, layers = 26, 26
    f = vqse_ising.build(n, layers, "f64")
    h = W.tfim_term(1.0)
    p = np.random.default_rng(42).normal(size=2 * layers)
    W.vqse_loss_and_grad(f, p, n, h)  # warm-up
    t0 = time.perf_counter()
    for _ in range(steps):
        e, _ = W.vqse_loss_and_grad(f, p, n, h)
    dt = (time.perf_counter() - t0) / steps
    return {"s_per_loss_grad_call": round(dt, 4), "energy": round(e, 6), "qubits": n,
            "layers": layers, "gates": 2 * n * layers, "dtype": "c128 (f64)",
            "calls": steps}


def micro(args):
    """Per-kernel bandwidth: each gate kind at every position, forward and fused reverse
    (single-gate kernels: fusion off)."""
    os.environ["QDC_FUSE"] = "0"
    import quantum_differentiable_circuit as q
    n, prec = args.qubits, args.precision
    dt = np.complex64 if prec == "f32" else np.complex128
    rng = np.random.default_rng(0)
    rows = []

    def run(label, setup):
        c = q.circuit_class(prec)(n)
        var = setup(c)
        c.forward([], var)  # warm-up
        c.backward(sigma_z_cotangents(1, dt), [], var)
        c.profile(True)
        for _ in range(3):
            c.forward([], var)
            c.backward(sigma_z_cotangents(1, dt), [], var)
        stats = c.profile_collect()
        c.profile(False)
        for k, s in stats.items():
            if s["total_ms"] > 0 and k not in ("finalize",):
                gbs = s["algo_bytes"] / (s["total_ms"] * 1e-3) / 1e9
                rows.append((label, k, s["launches"], s["total_ms"] / s["launches"], gbs))
                print(f"{label:14s} {k:18s} n={s['launches']:4d} {s['total_ms'] / s['launches']:8.3f} ms"
                      f" {gbs:8.1f} GB/s  {gbs / HBM_PEAK_GBS:6.1%}", flush=True)
        del c

    reps = 8
    for pos in range(n):
        def s1(c, pos=pos):
            for _ in range(reps):
                c.add_q1_var_gate(pos)
            c.get_q1_dens_op_with_grad(pos)
            return [np.ascontiguousarray(O_haar(rng, 2), dtype=dt) for _ in range(reps)]
        run(f"q1 {pos}", s1)
    for pos2, pos1 in [(0, 1), (1, 0), (5, 20), (26, 27), (27, 0), (1, 2), (3, 9), (14, 13)]:
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
    comm = None
    if world > 1:
        from quantum_differentiable_circuit.distributed import Communicator
        comm = Communicator(args.precision, device=local)
    c, ins, vg = build_circuit(q, n, args.layers, args.seed, args.precision, comm,
                               args.local_shards)
    ngates = len(vg)
    cots = sigma_z_cotangents(sum(1 for k, _ in ins if k in (12, 13)), c.dtype)
    remaps = 0
    shards = world if world > 1 else (args.local_shards or 1)
    if shards > 1:
        instr = [(k, *p) for k, p in ins]
        f_ops, end = q.plan(n, shards, instr, 1, precision=args.precision)
        b_ops, _ = q.plan(n, shards, instr, 2, start_phys=end, precision=args.precision)
        remaps = sum(o["type"] == "remap" for o in f_ops + b_ops)

    for _ in range(args.warmup):
        c.forward([], vg)
        c.backward(cots, [], vg)
    c.synchronize()

    c.profile(True)
    barrier(world)
    c.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dens = c.forward([], vg)
        grads = c.backward(cots, [], vg)
    c.synchronize()
    elapsed = time.perf_counter() - t0
    barrier(world)
    stats = c.profile_collect()
    c.profile(False)

    elapsed = max_over_ranks(elapsed, world)
    value = ngates * args.steps / elapsed  # the one sharded circuit's gate applications

    # dominant HBM kernel = the one with the largest share of measured device time
    dom_name, dom = max(((k, v) for k, v in stats.items() if k != "alltoall"),
                        key=lambda kv: kv[1]["total_ms"])
    avg_ms = dom["total_ms"] / dom["launches"]
    bytes_per_launch = dom["algo_bytes"] / dom["launches"]
    dom_flops = dom.get("algo_flops", 0.0) / dom["launches"]
    valu_peak = VALU_PEAK_TFLOPS[args.precision]
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    traffic = None
    pmc_path = Path(args.pmc) if args.pmc else ROOT / "profiles" / "pmc_traffic.json"
    if pmc_path.exists():
        try:
            traffic = json.loads(pmc_path.read_text()).get(dom_name)
        except Exception:  # noqa: BLE001
            traffic = None
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
    eff = ngates * 6 * state_bytes / (elapsed / args.steps) / 1e9 / max(world, 1)
    effective = {"per_gpu_GB/s": round(eff, 1), "x_hbm_peak": round(eff / HBM_PEAK_GBS, 3),
                 "definition": "gates x (2S fwd + 4S bwd) per step / step time, per GPU"}
    gate_kernels = dense_kernels = vqse = None
    if rank == 0 and world == 1 and not args.no_gate_sample:
        # auxiliary samples: a failure there is reported in the line, never loses the headline
        def aux(fn, *a):
            try:
                return fn(*a)
            except Exception as e:  # noqa: BLE001
                return {"error": f"{type(e).__name__}: {e}"[:300]}
        gate_kernels = aux(gate_kernel_sample, args, n)
        dense_kernels = aux(dense_gate_sample, args, n)
        vqse = aux(vqse_sample)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args, args.cpu_qubits or n)
        except Exception as e:  # noqa: BLE001
            cpu = {"error": f"{type(e).__name__}: {e}"[:300]}

    if rank == 0:
        state_gib = (1 << n) * (8 if args.precision == "f32" else 16) / 2**30
        line = {
            "metric": "gate-applications/sec (fwd+bwd) at n qubits",
            "value": round(value, 3),
            "unit": "gate-applications/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "c64 (f32)" if args.precision == "f32" else "c128 (f64)",
            "data": "synthetic (seeded Haar-random gates, |0..0> initial state)",
            "config": {"workload": f"C2 layered random circuit (configs[1] generator) at the "
                                   f"metric's n={n}, fwd+bwd",
                       "qubits": n, "layers": args.layers, "gates_per_step": ngates,
                       "densities_per_step": len(cots), "state_GiB": state_gib,
                       "parallelism": (f"state sharded over {world} GPUs by high qubits, "
                                       f"RCCL all-to-all remaps") if world > 1 else
                                      (f"rehearsal: {shards} shards on one GPU (device copies)"
                                       if shards > 1 else "single GPU"),
                       "remaps_per_step": remaps},
            "roofline": {"bound": "hbm", "kernel": dom_name, "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
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
            "effective_gate_bandwidth": effective,
            "gate_kernels": gate_kernels,
            "dense_gate_kernels": dense_kernels,
            "vqse_c3": vqse,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

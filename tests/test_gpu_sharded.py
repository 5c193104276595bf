"""GPU parity of the sharded state.

* `local_shards=G` runs the complete sharded data path (planner, pack kernel, block exchange,
  per-shard reductions + sum) with every shard on the one GPU: it must equal the oracle and
  the unsharded HIP path.
* With >= 2 GPUs, the RCCL transport runs one process per GPU (skipped on a 1-GPU box; the
  driver's multi-GPU bench exercises it)."""
import os
import socket

import numpy as np
import pytest

import floors as F
from oracle import oracle as O

pytestmark = pytest.mark.gpu
DT = {"f32": np.complex64, "f64": np.complex128}


def build(q, prec, n, ins, **kw):
    c = q.circuit_class(prec)(n, **kw)
    for kind, pos in ins:
        c._push(kind, *pos)
    return c


def normrel(a, b):
    a, b = np.asarray(a).reshape(-1), np.asarray(b).reshape(-1)
    return np.abs(a - b).max() / np.abs(b).max()


@pytest.mark.parametrize("prec", ["f32", "f64"])
@pytest.mark.parametrize("shards", [2, 4, 8])
def test_local_shards_match_oracle(prec, shards):
    import quantum_differentiable_circuit as q
    n = 11
    ins, const, var, _ = O.autodiff_circuit(n, 2, seed=17)
    psi0 = O.random_state(np.random.default_rng(2), n)
    fl = F.Floor(prec, n, ins, const, var, psi0=psi0, cots=F.tsallis_cots)
    c = build(q, prec, n, ins, local_shards=shards)
    c.set_state_from_vector(fl.psi0)
    what = f"autodiff n={n} {prec} {shards} shards "
    fl.check("run", c.run(fl.const, fl.var), what)
    fl.check("forward", c.forward(fl.const, fl.var), what)
    phys, world, _, nloc = c.layout()
    assert world == shards and nloc == shards
    fl.check("state", c.get_state(0), what)  # forward final state, un-permuted
    fl.check("grads", c.backward(fl.cots, fl.const, fl.var), what)
    fl.check("uncomputed", c.get_state(0), what)


def test_local_shards_equal_unsharded_on_brickwork():
    """Gates straddling the shard boundary every layer; sharded == unsharded HIP path."""
    import quantum_differentiable_circuit as q
    n = 16
    ins, var = O.layered_circuit(n, 3, seed=33)
    fl = F.Floor("f32", n, ins, [], var, run=False)
    a = build(q, "f32", n, ins)
    b = build(q, "f32", n, ins, local_shards=8)
    da, db = a.forward([], fl.var), b.forward([], fl.var)
    fl.check("forward", db, "C2 n=16 8 shards ")
    F.check_pair("f32", db, da, fl.floor["forward"], "C2 n=16 8 shards vs unsharded forward")
    ga, gb = a.backward(fl.cots, [], fl.var), b.backward(fl.cots, [], fl.var)
    fl.check("grads", gb, "C2 n=16 8 shards ")
    F.check_pair("f32", gb, ga, fl.floor["grads"], "C2 n=16 8 shards vs unsharded grads")

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rccl_worker(rank, world, port, q_out):
    os.environ["LOCAL_RANK"] = str(rank)
    try:
        import quantum_differentiable_circuit as q
        from quantum_differentiable_circuit.distributed import Communicator
        comm = Communicator("f64", rank=rank, world=world,
                            id_file=f"/tmp/qdc_test_rccl_{port}.id")
        n = 12
        ins, var = O.layered_circuit(n, 2, seed=7)
        c = build(q, "f64", n, ins, comm=comm)
        d = c.forward([], var)
        g = c.backward([np.diag([1.0, -1.0]).astype(np.complex128) for _ in d], [], var)
        q_out.put((rank, d, g, None))
    except Exception:  # noqa: BLE001
        import traceback
        q_out.put((rank, None, None, traceback.format_exc()))


def test_rccl_two_processes():
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs >= 2 GPUs (RCCL needs one GPU per rank)")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q_out = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rccl_worker, args=(r, 2, port, q_out)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q_out.get(timeout=300) for _ in range(2)]
    for p in ps:
        p.join(timeout=60)
    for r in res:
        assert r[3] is None, r[3]
    n = 12
    ins, var = O.layered_circuit(n, 2, seed=7)
    o = O.OracleCircuit(n)
    for kind, pos in ins:
        o.add(kind, *pos)
    dens = o.forward([], var)
    grads = o.backward([np.diag([1.0, -1.0]) for _ in dens], [], var)
    for _, d, g, _ in res:
        assert max(np.abs(a - b).max() for a, b in zip(d, dens)) < 1e-11
        assert normrel(np.concatenate(g), np.concatenate(grads)) < 1e-10


def test_devices_multi_stream_one_gpu():
    """qdc_circuit_new_devices with one device repeated: every shard on its own stream and
    context (program copy, reduction arena), exchanged by copies ordered with events — the
    single-process multi-GPU plumbing minus RCCL, on one GPU; equal to the oracle within 4x the
    floor and to the single-stream loopback shards."""
    import quantum_differentiable_circuit as q
    n = 14
    ins, var = O.layered_circuit(n, 4, seed=41)
    fl = F.Floor("f32", n, ins, [], var, run=False)
    for devs in ([0], [0, 0], [0, 0, 0, 0]):
        c = build(q, "f32", n, ins, devices=devs)
        d = c.forward([], fl.var)
        fl.check("forward", d, f"C2 n={n} devices={devs} ")
        fl.check("state", c.get_state(0), f"C2 n={n} devices={devs} ")
        g = c.backward(fl.cots, [], fl.var)
        fl.check("grads", g, f"C2 n={n} devices={devs} ")
        fl.check("uncomputed", c.get_state(0), f"C2 n={n} devices={devs} ")
        phys, world, _, nloc = c.layout()
        assert world == len(devs) and nloc == len(devs)
        if len(devs) > 1:
            ref = build(q, "f32", n, ins, local_shards=len(devs))
            dr = ref.forward([], fl.var)
            F.check_pair("f32", d, dr, fl.floor["forward"], f"devices={devs} vs local shards")
            F.check_pair("f32", g, ref.backward(fl.cots, [], fl.var), fl.floor["grads"],
                         f"devices={devs} vs local shards grads")


def test_devices_rccl_single_process():
    """One process, one shard per GPU (ncclCommInitAll); skipped on a 1-GPU box (the driver's
    multi-GPU bench runs bench.py --gpus N)."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs >= 2 GPUs")
    import quantum_differentiable_circuit as q
    n = 14
    ins, var = O.layered_circuit(n, 3, seed=43)
    fl = F.Floor("f64", n, ins, [], var, run=False)
    c = build(q, "f64", n, ins, devices=2)
    fl.check("forward", c.forward([], fl.var), "devices=2 ")
    fl.check("grads", c.backward(fl.cots, [], fl.var), "devices=2 ")


def _hip():
    """The HIP runtime instance the circuit library is bound to.  torch bundles its own copy with
    the same soname: loaded first, it is the one libqdc binds (ROCm's is then never mapped), else
    libqdc maps ROCm's through its RUNPATH.  A bare dlopen("libamdhip64.so") may instead open a
    second instance with its own device state."""
    import ctypes
    from quantum_differentiable_circuit import _native
    _native.load("f32")
    mapped = []
    for line in open("/proc/self/maps"):
        path = line.split()[-1]
        if "libamdhip64" in path and path not in mapped:
            mapped.append(path)
    if not mapped:
        raise RuntimeError("no HIP runtime is mapped")
    own = [p for p in mapped if "/torch/" not in p]
    return ctypes.CDLL((own or mapped)[0])


def _current_device():
    import ctypes
    d = ctypes.c_int(-1)
    assert _hip().hipGetDevice(ctypes.byref(d)) == 0
    return d.value


def _set_device(i):
    import ctypes
    assert _hip().hipSetDevice(ctypes.c_int(i)) == 0


def _device_count():
    import ctypes
    n = ctypes.c_int(0)
    assert _hip().hipGetDeviceCount(ctypes.byref(n)) == 0
    return n.value


def test_entry_points_keep_the_callers_device():
    """Every circuit entry point leaves the caller's HIP device current (qdc::DeviceGuard): a
    multi-device circuit switches devices per shard, and the C-ABI primitives, torch and the
    caller's code must not find themselves on the last shard's GPU afterwards.  On one GPU the
    repeated-device circuit covers the per-shard contexts; with two GPUs the circuit lives on
    device 1 while the caller stays on device 0 (and the reverse)."""
    import quantum_differentiable_circuit as q
    n = 10
    ins, var = O.layered_circuit(n, layers=1, seed=3)
    vg = [np.ascontiguousarray(g, dtype=np.complex64) for g in var]
    cots = F.sigma_z_cots([np.zeros((2, 2))] * n, np.complex64)
    cases = [([0, 0], 0)]
    if _device_count() >= 2:
        cases += [([1], 0), ([0], 1), ([0, 1], 1)]
    for devs, caller in cases:
        _set_device(caller)
        c = build(q, "f32", n, ins, devices=devs)
        assert _current_device() == caller, f"constructor moved the caller ({devs})"
        c.forward([], vg)
        c.backward(cots, [], vg)
        c.get_state(0)
        c.synchronize()
        assert _current_device() == caller, f"forward/backward moved the caller ({devs})"
        del c
        assert _current_device() == caller, f"destructor moved the caller ({devs})"
    _set_device(0)


@pytest.mark.parametrize("prec,kw", [("f32", {"local_shards": 4}), ("f32", {"devices": [0, 0]}),
                                     ("f64", {"local_shards": 4})])
def test_specialized_passes_sharded(prec, kw):
    """Sharded circuits run the passes specialized per program too (csrc/qdc_spec.hpp; every
    shard the same program, the kernel loaded on each shard's device): forced on (QDC_SPEC=2)
    they match the interpreted kernels — f32 bit-identical, f64 within 1e-14 (two FMA
    contractions of a complex product, tests/test_gpu_fusion.py) — and the oracle's floors."""
    import quantum_differentiable_circuit as q
    n = 18
    ins, var = O.layered_circuit(n, 3, seed=41)
    fl = F.Floor(prec, n, ins, [], var, run=False)
    out = {}
    for mode in ("0", "2"):
        old = os.environ.get("QDC_SPEC")
        os.environ["QDC_SPEC"] = mode
        try:
            c = build(q, prec, n, ins, **kw)
        finally:
            if old is None:
                del os.environ["QDC_SPEC"]
            else:
                os.environ["QDC_SPEC"] = old
        launched = q.jit_stats(prec)["launched"]
        d = c.forward([], fl.var)
        g = c.backward(fl.cots, [], fl.var)
        c.synchronize()
        ran = q.jit_stats(prec)["launched"] - launched
        assert (ran > 0) == (mode == "2"), (mode, ran, q.jit_stats(prec))
        what = f"C2 n={n} {prec} {kw} spec={mode} "
        fl.check("forward", d, what)
        fl.check("grads", g, what)
        out[mode] = (np.asarray(d).reshape(-1),
                     np.concatenate([np.asarray(x).reshape(-1) for x in g]))
    for k, name in enumerate(("densities", "grads")):
        a0, a2 = out["0"][k], out["2"][k]
        if prec == "f32":
            assert np.array_equal(a0, a2), f"{kw}: specialized {name} differ"
        else:
            rel = np.linalg.norm(a2 - a0) / max(np.linalg.norm(a0), 1e-300)
            assert rel <= 1e-14, f"{kw}: specialized {name} differ by {rel:.2e}"


@pytest.mark.parametrize("shards", [2, 8])
def test_tiled_pack_equals_direct_pack(shards):
    """The remap's pack / unpack through LDS tiles (k_pack_tile: whole-wave accesses whatever the
    victims) is the same permutation as the direct kernel (k_pack): a deep random circuit whose
    remaps pick low victims, on local shards, gives bit-identical densities, gradients and
    states with QDC_PACK_TILE=0 and 1 (a process reads the knob once: two child processes)."""
    import json
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    n = 18
    code = f"""
import sys, numpy as np
sys.path[:0] = [{str(root)!r}, {str(root / 'differentiable-quantum-circuit-cuda_amd')!r}]
import quantum_differentiable_circuit as q
from quantum_differentiable_circuit import workloads as W
ins, var = W.deep_random_circuit({n}, 600, seed=71)
c = q.circuit_class("f32")({n}, local_shards={shards})
for kind, pos in ins:
    c._push(kind, *pos)
vg = [np.ascontiguousarray(g, dtype=np.complex64) for g in var]
d = c.forward([], vg)
g = c.backward([np.diag([1.0, -1.0]).astype(np.complex64) for _ in d], [], vg)
np.savez(sys.argv[1], d=np.concatenate([x.reshape(-1) for x in d]), g=np.concatenate(g),
         f=c.get_state(0), b=c.get_state(2))
"""
    import tempfile
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for tile in ("0", "1"):
            env = dict(os.environ, QDC_PACK_TILE=tile)
            path = f"{td}/o{tile}.npz"
            r = subprocess.run([sys.executable, "-c", code, path], env=env, capture_output=True,
                               text=True, timeout=300)
            assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
            z = np.load(path)
            out[tile] = {k: z[k] for k in z.files}
    for k in out["0"]:
        assert np.array_equal(out["0"][k], out["1"][k]), f"{shards} shards: {k} differs"
    ins, _ = __import__("quantum_differentiable_circuit.workloads", fromlist=["x"]).deep_random_circuit(n, 600, seed=71)
    import quantum_differentiable_circuit as q
    ops, _ = q.plan(n, shards, [(k, *p) for k, p in ins], 3, precision="f32")
    low = [o["victims"] for o in ops if o["type"] == "remap" and o["pack"] and min(o["victims"]) < 10]
    print(f"[pack] {shards} shards: {len(low)} remaps with victims below chunk bit 9; tiled == direct")
    assert low, "the case must exercise low victims"

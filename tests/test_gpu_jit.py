"""The specialized-kernel JIT beyond one call's own compile (csrc/qdc_jit.hpp, round 5):

* ahead-of-time compilation (qdc_precompile, what build() runs for the bench's programs): a
  host-only dry run of the runtime's plans, schedules and pass programs must name exactly the
  kernels the real calls launch, so a process running the circuit afterwards compiles nothing;
* the background compiler: a program with more distinct kernels than QDC_SPEC_MAX (deep random
  circuits, config C5) runs its passes on the generic kernels while the missing ones compile
  in a background thread, and launches the specialized ones once they exist — with results
  bit-identical to the generic kernels' in f32.

Each case runs in a child process with its own cache directory (a process picks its directory
once), and checks its results against the oracle's floors."""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

import floors as F
from oracle import oracle as O

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent
DT = {"f32": np.complex64, "f64": np.complex128}

CHILD = """
import json, sys
import numpy as np
sys.path[:0] = [{root!r}, {pkg!r}]
import quantum_differentiable_circuit as q
from oracle import oracle as O
prec, mode, n, layers, world, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), sys.argv[6]
dt = np.complex64 if prec == "f32" else np.complex128
if layers > 0:
    ins, var = O.layered_circuit(n, layers, seed=61)
    const = []
else:
    ins, const, var = O.random_circuit(n, 240, seed=62, density_every=4)
cg = [np.ascontiguousarray(g, dtype=dt) for g in const]
vg = [np.ascontiguousarray(g, dtype=dt) for g in var]
z = np.load(out + "_cots.npz")
cots = [np.ascontiguousarray(z[f"arr_{{i}}"], dtype=dt) for i in range(len(z.files))]
res = {{}}
if mode == "precompile":
    instr = [(k, *p) for k, p in ins]
    res["kernels"] = q.precompile(n, instr, cg, vg, cots, world=world, precision=prec)
else:
    c = q.circuit_class(prec)(n, local_shards=world if world > 1 else None)
    for kind, pos in ins:
        c._push(kind, *pos)
    calls = []
    for call in range(2 if mode == "background" else 1):
        before = q.jit_stats(prec)["launched"]
        d = c.forward(cg, vg)
        g = c.backward(cots, cg, vg)
        c.synchronize()
        st = q.jit_stats(prec)
        calls.append({{"launched": st["launched"] - before, "queued": st["queued"]}})
        np.save(out + f"_d{{call}}.npy", np.concatenate([np.asarray(x).reshape(-1) for x in d]))
        np.save(out + f"_g{{call}}.npy", np.concatenate([np.asarray(x).reshape(-1) for x in g]))
        if mode == "background" and call == 0:
            res["left_after_wait"] = q.jit_wait(600.0, prec)
    res["calls"] = calls
res["stats"] = q.jit_stats(prec)
print(json.dumps(res))
"""


def _child(tmp_path, env, *args):
    code = CHILD.format(root=str(ROOT), pkg=str(ROOT / "differentiable-quantum-circuit-cuda_amd"))
    e = dict(os.environ, **env)
    e.pop("QDC_LIB_DIR", None)
    r = subprocess.run([sys.executable, "-c", code, *map(str, args)], env=e, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def _floor(prec, n, layers, tmp_path, tag):
    if layers > 0:
        ins, var = O.layered_circuit(n, layers, seed=61)
        const = []
    else:
        ins, const, var = O.random_circuit(n, 240, seed=62, density_every=4)
    fl = F.Floor(prec, n, ins, const, var, run=False)
    np.savez(tmp_path / f"{tag}_cots.npz", *fl.cots)
    return fl


@pytest.mark.parametrize("prec,layers,world", [("f32", 3, 1), ("f32", 0, 1), ("f32", 3, 4),
                                               ("f64", 3, 1)])
def test_precompiled_programs_compile_nothing(tmp_path, prec, layers, world):
    """qdc_precompile's dry run names exactly the kernels the real calls need: a process that
    then runs the circuit from the same cache directory compiles none, launches specialized
    passes, and is within the oracle's floors (unsharded and 4 local shards, layered and random
    circuits with densities between the gates)."""
    n = 14
    tag = f"{prec}_{layers}_{world}"
    fl = _floor(prec, n, layers, tmp_path, tag)
    jit = tmp_path / "jit"
    jit.mkdir(mode=0o700)
    env = {"QDC_SPEC": "2", "QDC_SPEC_MAX": "100000", "QDC_JIT_DIR": str(jit), "QDC_JIT_PREBUILT": "0"}
    pre = _child(tmp_path, env, prec, "precompile", n, layers, world, tmp_path / tag)
    assert pre["kernels"] > 0 and pre["stats"]["compiled"] == pre["kernels"], pre
    run = _child(tmp_path, env, prec, "run", n, layers, world, tmp_path / tag)
    print(f"[jit] precompiled {tag}: {pre['kernels']} kernels; run {run}")
    assert run["stats"]["compiled"] == 0, f"the dry run missed kernels: {run}"
    assert run["calls"][0]["launched"] > 0, run
    what = f"precompiled {tag} "
    fl.check("forward", np.load(tmp_path / f"{tag}_d0.npy"), what)
    fl.check("grads", np.load(tmp_path / f"{tag}_g0.npy"), what)


def test_background_jit_for_deep_programs(tmp_path):
    """More distinct kernels than QDC_SPEC_MAX: the first call runs its passes generic and queues
    the kernels for the background compiler (a kernel the compiler finishes during the call — a
    backward pass sharing a forward pass's program — may already launch); after jit_wait the
    second call launches specialized passes, bit-identical to the first call's (f32), within the
    oracle's floors."""
    n, prec = 14, "f32"
    tag = "bg"
    fl = _floor(prec, n, 0, tmp_path, tag)
    jit = tmp_path / "jit"
    jit.mkdir(mode=0o700)
    env = {"QDC_SPEC": "2", "QDC_SPEC_MAX": "2", "QDC_JIT_DIR": str(jit), "QDC_JIT_PREBUILT": "0"}
    res = _child(tmp_path, env, prec, "background", n, 0, 1, tmp_path / tag)
    print(f"[jit] background: {res}")
    c0, c1 = res["calls"]
    assert res["stats"]["compiled"] > 0 and c0["launched"] < c1["launched"] // 4, res
    assert res["left_after_wait"] == 0 and c1["launched"] > 0, res
    for k in ("d", "g"):
        a, b = np.load(tmp_path / f"{tag}_{k}0.npy"), np.load(tmp_path / f"{tag}_{k}1.npy")
        assert np.array_equal(a, b), f"specialized call differs from the generic one ({k})"
    fl.check("forward", np.load(tmp_path / f"{tag}_d1.npy"), "background-jit ")
    fl.check("grads", np.load(tmp_path / f"{tag}_g1.npy"), "background-jit ")

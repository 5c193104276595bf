#!/usr/bin/env python3
"""Specialized vs interpreted reverse passes on one circuit: which outputs differ, by how much,
and whether each mode is deterministic (GPU debugging aid for tests/test_gpu_fusion.py)."""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "tests", ROOT / "differentiable-quantum-circuit-cuda_amd"):
    sys.path.insert(0, str(p))
import floors as F  # noqa: E402
from oracle import oracle as O  # noqa: E402


def run(mode, n, ins, fl):
    import quantum_differentiable_circuit as q
    os.environ["QDC_SPEC"] = mode
    c = q.circuit_class("f32")(n)
    for kind, pos in ins:
        c._push(kind, *pos)
    d = c.forward(fl.const, fl.var)
    g = c.backward(fl.cots, fl.const, fl.var)
    flat = lambda xs: np.concatenate([np.asarray(x).reshape(-1) for x in xs])
    return flat(d), flat(g), np.asarray(c.get_state(0)).reshape(-1), np.asarray(c.get_state(2)).reshape(-1)


n = int(sys.argv[1]) if len(sys.argv) > 1 else 14
layers = int(sys.argv[2]) if len(sys.argv) > 2 else 4
ins, var = O.layered_circuit(n, layers, seed=31)
fl = F.Floor("f32", n, ins, [], var, run=False)
a = run("0", n, ins, fl)
b = run("2", n, ins, fl)
c = run("2", n, ins, fl)
for k, name in enumerate(("dens", "grads", "fwd", "bwd")):
    x, y, z = a[k].reshape(-1), b[k].reshape(-1), c[k].reshape(-1)
    dif = np.nonzero(x != y)[0]
    print(f"{name}: spec vs interp differ at {len(dif)} of {x.size}, max |d| {np.abs(x - y).max():.3e}, "
          f"spec repeat identical {np.array_equal(y, z)}, first idx {dif[:8]}")

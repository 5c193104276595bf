#!/usr/bin/env python3
"""Densities, gradients and both final states of one C2 forward + backward (n = 22: specialized
passes on) with the library QDC_LIB_DIR selects, saved to argv[1] (.npz): library variants that
only reorder or re-encode the same floating-point operations must agree bit for bit."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "differentiable-quantum-circuit-cuda_amd")]
import quantum_differentiable_circuit as q  # noqa: E402
from quantum_differentiable_circuit import workloads as W  # noqa: E402

n = 22
ins, var = W.layered_circuit(n, 4, 24)
c = q.circuit_class("f32")(n)
for kind, pos in ins:
    c._push(kind, *pos)
vg = [np.ascontiguousarray(g, dtype=np.complex64) for g in var]
d = c.forward([], vg)
g = c.backward([np.diag([1.0, -1.0]).astype(np.complex64) for _ in d], [], vg)
# (the states as 64-bit hashes of their bytes: gpurun_out/ must stay small)
import hashlib  # noqa: E402
h = lambda a: np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest()[:8], np.uint64)
np.savez(sys.argv[1], d=np.concatenate([x.reshape(-1) for x in d]), g=np.concatenate(g),
         f=h(c.get_state(0)), b=h(c.get_state(2)))
print("saved", sys.argv[1], q.jit_stats("f32"))

#!/usr/bin/env python3
"""Which part of the fused runtime sets the uncompute error of config C5 at depth (GPU, f32):
the same 10 000-gate circuit at n = 14 (tests/test_gpu_drift.py) through runtime variants
chosen by environment knobs read at circuit construction (QDC_FUSE, QDC_RQ, QDC_RQ_PERM, ...),
each error against the complex128 oracle and the reference algorithm's own f32 floor.
usage: python3 tools/drift_ab.py [f32|f64] [n] [gates]"""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "tests", ROOT / "differentiable-quantum-circuit-cuda_amd"):
    sys.path.insert(0, str(p))

import floors as F  # noqa: E402
from quantum_differentiable_circuit import workloads as W  # noqa: E402

VARIANTS = [
    ("default", {}),
    ("unfused (single-gate kernels)", {"QDC_FUSE": "0"}),
    ("fused, LDS passes (no register-resident)", {"QDC_RQ": "0"}),
    ("fused, no permuting passes", {"QDC_RQ_PERM": "0"}),
    ("fused, one gate per pass op", {"QDC_FUSE_MAX_OPS": "1"}),
    ("fused, plain state layout", {"QDC_STATE_ILV": "0"}),
    ("fused, no densities in passes", {"QDC_FUSE_MEAS": "0"}),
]


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "f32"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 14
    ng = int(sys.argv[3]) if len(sys.argv) > 3 else 10000
    ins, var = W.deep_random_circuit(n, ng, seed=33)
    fl = F.Floor(prec, n, ins, [], var, run=False)
    print(f"C5 n={n} {ng} gates {prec}: floors " + " ".join(f"{k} {v:.3e}" for k, v in fl.floor.items()),
          flush=True)
    import quantum_differentiable_circuit as q
    for name, env in VARIANTS:
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            c = q.circuit_class(prec)(n)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        for kind, pos in ins:
            c._push(kind, *pos)
        dens = c.forward([], fl.var)
        st = c.get_state(0)
        g = c.backward(fl.cots, [], fl.var)
        un = c.get_state(0)
        row = {"forward": F.normrel(dens, fl.exact["forward"]), "state": F.normrel(st, fl.exact["state"]),
               "grads": F.normrel(g, fl.exact["grads"]), "uncomputed": F.normrel(un, fl.exact["uncomputed"])}
        print(f"{name:42s} " + " ".join(f"{k} {v:.3e} ({v / fl.floor[k]:.2f}x)" for k, v in row.items()),
              flush=True)
        del c


if __name__ == "__main__":
    main()

"""Gate constants of the reference's test fixtures (src/common_gates.rs:19-34), in the
precision of a build: `get_hadamard()` (4 entries) and `get_cnot()` (16 entries), row-major
U[out, in] flattened as every gate buffer of the C ABI (include/qdc/primitives.h).  The CNOT's
control is the two-qubit gate's first position (pos2, the MSB of its local index,
src/qdc/circuit.py:27-28).

As in the Rust module, 1/sqrt(2) is formed in the build's own float type (f32: 1.0f / sqrtf(2)).
"""
from __future__ import annotations

import numpy as np

from ._native import PRECISIONS, default_precision

__all__ = ["get_hadamard", "get_cnot"]

_REAL = {"f32": np.float32, "f64": np.float64}


def _prec(precision):
    p = precision or default_precision()
    if p not in PRECISIONS:
        raise ValueError(f"precision must be one of {sorted(PRECISIONS)}, got {p!r}")
    return p


def get_hadamard(precision: str | None = None) -> np.ndarray:
    """[1, 1; 1, -1] / sqrt(2) (common_gates.rs:19-25)."""
    p = _prec(precision)
    r = _REAL[p]
    s = r(1.0) / np.sqrt(r(2.0))
    return np.array([s, s, s, -s], dtype=PRECISIONS[p])


def get_cnot(precision: str | None = None) -> np.ndarray:
    """Identity on |00>, |01>; swaps |10> and |11> (common_gates.rs:27-34)."""
    p = _prec(precision)
    return np.array([1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 0, 1, 0, 0, 1, 0], dtype=PRECISIONS[p])

"""ctypes op table over oracle/cpu_ref.c — TEST INFRASTRUCTURE ONLY (see oracle/oracle.py).

`CRefOps(precision)` plugs the C/OpenMP restatement of the reference's CUDA kernels
(src/primitives.cu:176-953, index rules verbatim) into `oracle.OracleCircuit`; states stay in
the build's precision (complex64 / complex128) and are updated in place, like device states.
bench.py times it as the CPU baseline ("kind": "port").
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

BUILD = Path(__file__).resolve().parent / "build"
_LIBS = {}


def _lib(precision):
    if precision not in _LIBS:
        path = BUILD / f"libcref_{precision}.so"
        if not path.exists():
            raise ImportError(f"{path} not built (make -C oracle)")
        lib = C.CDLL(str(path))
        P, S = C.c_void_p, C.c_size_t
        for name, args in {
            "cref_q1gate": [P, P, S, S], "cref_q2gate": [P, P, S, S, S],
            "cref_q2gate_diag": [P, P, S, S, S], "cref_q1density": [P, P, S, S],
            "cref_q2density": [P, P, S, S, S], "cref_q1grad": [P, P, P, S, S],
            "cref_q2grad": [P, P, P, S, S, S], "cref_q2grad_diag": [P, P, P, S, S, S],
            "cref_set2standard": [P, S], "cref_copy": [P, P, S],
            "cref_conj_and_double": [P, P, S], "cref_add": [P, P, S],
        }.items():
            fn = getattr(lib, name)
            fn.restype = None
            fn.argtypes = args
        lib.cref_threads.restype = C.c_int
        lib.cref_set_threads.restype = None
        lib.cref_set_threads.argtypes = [C.c_int]
        _LIBS[precision] = lib
    return _LIBS[precision]


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class CRefOps:
    def __init__(self, precision="f32"):
        self.lib = _lib(precision)
        self.state_dtype = np.dtype(np.complex64 if precision == "f32" else np.complex128)

    def threads(self):
        return int(self.lib.cref_threads())

    def set_threads(self, t):
        self.lib.cref_set_threads(int(t))

    def _n(self, s):
        return s.size.bit_length() - 1

    def _g(self, g):
        return np.ascontiguousarray(g, dtype=self.state_dtype).reshape(-1)

    def apply_q1_gate(self, s, g, pos):
        g = self._g(g)
        self.lib.cref_q1gate(_p(s), _p(g), pos, self._n(s))
        return s

    def apply_q2_gate(self, s, g, pos2, pos1):
        g = self._g(g)
        self.lib.cref_q2gate(_p(s), _p(g), pos2, pos1, self._n(s))
        return s

    def apply_q2_gate_diag(self, s, g, pos2, pos1):
        g = self._g(g)
        self.lib.cref_q2gate_diag(_p(s), _p(g), pos2, pos1, self._n(s))
        return s

    def get_q1_density(self, s, pos):
        out = np.zeros(4, self.state_dtype)
        self.lib.cref_q1density(_p(s), _p(out), pos, self._n(s))
        return out

    def get_q2_density(self, s, pos2, pos1):
        out = np.zeros(16, self.state_dtype)
        self.lib.cref_q2density(_p(s), _p(out), pos2, pos1, self._n(s))
        return out

    def get_q1_grad(self, f, b, pos):
        out = np.zeros(4, self.state_dtype)
        self.lib.cref_q1grad(_p(f), _p(b), _p(out), pos, self._n(f))
        return out

    def get_q2_grad(self, f, b, pos2, pos1):
        out = np.zeros(16, self.state_dtype)
        self.lib.cref_q2grad(_p(f), _p(b), _p(out), pos2, pos1, self._n(f))
        return out

    def get_q2_grad_diag(self, f, b, pos2, pos1):
        out = np.zeros(4, self.state_dtype)
        self.lib.cref_q2grad_diag(_p(f), _p(b), _p(out), pos2, pos1, self._n(f))
        return out

    def conj_and_double(self, s):
        out = np.empty_like(s)
        self.lib.cref_conj_and_double(_p(s), _p(out), self._n(s))
        return out

    def add(self, src, dst):
        self.lib.cref_add(_p(src), _p(dst), self._n(src))
        return dst

    def copy(self, s):
        out = np.empty_like(s)
        self.lib.cref_copy(_p(s), _p(out), self._n(s))
        return out

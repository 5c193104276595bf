"""ctypes bindings of the HIP hot-path library (libqdc_f32.so / libqdc_f64.so).

The C ABI is declared in ``include/qdc/primitives.h`` (the reference's 18 primitives,
``src/primitives_bind.rs:15-119``) and ``include/qdc/circuit.h`` (the circuit runtime that
replaces ``src/circuit.rs`` / ``src/quantized_tensor.rs``).  There is no fallback: if the
library is missing the import fails loudly, and every call that needs a GPU raises the HIP
error the library reports.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

PKG_ROOT = Path(__file__).resolve().parent.parent
LIB_DIR = PKG_ROOT / "lib"

PRECISIONS = {"f32": np.complex64, "f64": np.complex128}

# every symbol the headers declare (checked by tests/test_abi.py)
PRIMITIVES = (
    "set2standard", "get_state", "drop_state", "copy_to_host", "set_from_host", "q1gate",
    "q1gate_inv", "q2gate", "q2gate_inv", "q2gate_diag", "get_q1density", "get_q2density",
    "q1grad", "q2grad", "q2grad_diag", "conj_and_double", "add", "copy",
)
RUNTIME = (
    "qdc_circuit_new", "qdc_circuit_free", "qdc_circuit_qubits",
    "qdc_circuit_set_state_from_vector", "qdc_circuit_push", "qdc_circuit_len",
    "qdc_circuit_output_size", "qdc_circuit_grad_size", "qdc_circuit_execute",
    "qdc_circuit_backward", "qdc_circuit_get_state", "qdc_circuit_sync", "qdc_circuit_profile",
    "qdc_circuit_profile_collect", "qdc_circuit_host_times", "qdc_build_info", "qdc_comm_unique_id", "qdc_comm_init",
    "qdc_comm_free", "qdc_comm_allreduce", "qdc_circuit_gather_state", "qdc_circuit_new_sharded", "qdc_circuit_new_local_shards",
    "qdc_circuit_new_devices",
    "qdc_circuit_layout", "qdc_circuit_get_shard", "qdc_circuit_get_range", "qdc_plan", "qdc_fusion_schedule",
    "qdc_rq_plan", "qdc_spec_selftest", "qdc_gate_plan", "qdc_lane_plan", "qdc_qkgate", "qdc_abi_sync", "qdc_abi_profile", "qdc_abi_profile_collect",
    "qdc_jit_stats", "qdc_jit_dir", "qdc_spec_fingerprint", "qdc_spec_selftest_batch",
    "qdc_jit_wait", "qdc_precompile", "qdc_check_schedule", "qdc_trace_program",
)


class PanicException(BaseException):
    """Raised where the reference's Rust code panics (PyO3 surfaces those as
    ``pyo3_runtime.PanicException``, a ``BaseException``)."""


class PlanOp(C.Structure):
    """qdc_plan_op (include/qdc/circuit.h)."""
    _fields_ = [("type", C.c_int), ("instr", C.c_int), ("pos2", C.c_uint), ("pos1", C.c_uint),
                ("victims", C.c_uint * 8), ("nvictims", C.c_uint), ("pack", C.c_int)]


class KernelStat(C.Structure):
    _fields_ = [("name", C.c_char * 32), ("launches", C.c_size_t), ("total_ms", C.c_double),
                ("algo_bytes", C.c_double), ("algo_flops", C.c_double)]


_P = C.c_void_p
_S = C.c_size_t
_E = C.c_char_p  # const char* error (NULL = ok)


def _proto(lib):
    sig = {
        "set2standard": (None, [_P, _S]),
        "get_state": (_E, [C.POINTER(_P), _S]),
        "drop_state": (_E, [_P]),
        "copy_to_host": (_E, [_P, _P, _S]),
        "set_from_host": (_E, [_P, _P, _S]),
        "q1gate": (_E, [_P, _P, _S, _S]),
        "q1gate_inv": (_E, [_P, _P, _S, _S]),
        "q2gate": (_E, [_P, _P, _S, _S, _S]),
        "q2gate_inv": (_E, [_P, _P, _S, _S, _S]),
        "q2gate_diag": (_E, [_P, _P, _S, _S, _S]),
        "get_q1density": (_E, [_P, _P, _S, _S]),
        "get_q2density": (_E, [_P, _P, _S, _S, _S]),
        "q1grad": (_E, [_P, _P, _P, _S, _S]),
        "q2grad": (_E, [_P, _P, _P, _S, _S, _S]),
        "q2grad_diag": (_E, [_P, _P, _P, _S, _S, _S]),
        "conj_and_double": (None, [_P, _P, _S]),
        "add": (None, [_P, _P, _S]),
        "copy": (None, [_P, _P, _S]),
        "qdc_circuit_new": (_E, [C.POINTER(_P), _S]),
        "qdc_circuit_free": (None, [_P]),
        "qdc_circuit_qubits": (_S, [_P]),
        "qdc_circuit_set_state_from_vector": (_E, [_P, _P, _S]),
        "qdc_circuit_push": (_E, [_P, C.c_int, _S, _S]),
        "qdc_circuit_len": (_S, [_P]),
        "qdc_circuit_output_size": (_S, [_P, C.c_int]),
        "qdc_circuit_grad_size": (_S, [_P]),
        "qdc_circuit_execute": (_E, [_P, C.c_int, _P, _P, _S, _P, _P, _S, _P]),
        "qdc_circuit_backward": (_E, [_P, _P, _P, _S, _P, _P, _S, _P, _P, _S, _P]),
        "qdc_circuit_get_state": (_E, [_P, C.c_int, _P, _S]),
        "qdc_circuit_sync": (_E, [_P]),
        "qdc_circuit_profile": (_E, [_P, C.c_int]),
        "qdc_circuit_profile_collect": (_S, [_P, C.POINTER(KernelStat), _S]),
        "qdc_circuit_host_times": (_S, [_P, C.POINTER(C.c_double), _S, C.c_int]),
        "qdc_build_info": (C.c_char_p, []),
        "qdc_comm_unique_id": (_E, [C.c_char_p]),
        "qdc_comm_init": (_E, [C.POINTER(_P), C.c_int, C.c_int, C.c_char_p]),
        "qdc_comm_free": (None, [_P]),
        "qdc_comm_allreduce": (_E, [_P, C.POINTER(C.c_double), C.c_int, C.c_int]),
        "qdc_circuit_gather_state": (_E, [_P, C.c_int, _P, _S]),
        "qdc_circuit_new_sharded": (_E, [C.POINTER(_P), _S, _P]),
        "qdc_circuit_new_local_shards": (_E, [C.POINTER(_P), _S, C.c_int]),
        "qdc_circuit_new_devices": (_E, [C.POINTER(_P), _S, C.c_int, C.POINTER(C.c_int)]),
        "qdc_circuit_layout": (_E, [_P, C.POINTER(C.c_uint), C.POINTER(C.c_int),
                                    C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        "qdc_circuit_get_shard": (_E, [_P, C.c_int, C.c_int, _P, _S]),
        "qdc_circuit_get_range": (_E, [_P, C.c_int, C.c_int, _S, _P, _S]),
        "qdc_plan": (_S, [_S, _S, C.POINTER(C.c_int), C.POINTER(C.c_uint), C.POINTER(C.c_uint),
                          _S, C.c_int, C.POINTER(C.c_uint), C.POINTER(PlanOp), _S,
                          C.POINTER(C.c_uint)]),
        "qdc_fusion_schedule": (_S, [_S, C.c_int, _S, C.POINTER(C.c_int), C.POINTER(C.c_ubyte),
                                     _S, C.POINTER(PlanOp), _S, C.c_int, C.c_int,
                                     C.POINTER(C.c_uint), _S, C.POINTER(C.c_uint), _S,
                                     C.POINTER(C.c_uint), _S]),
        "qdc_qkgate": (_E, [_P, _P, C.POINTER(C.c_size_t), _S, _S]),
        "qdc_abi_sync": (_E, []),
        "qdc_abi_profile": (_E, [C.c_int]),
        "qdc_abi_profile_collect": (_S, [C.POINTER(KernelStat), _S]),
        "qdc_gate_plan": (C.c_int, [C.c_uint, C.c_uint, C.c_uint, C.c_uint, C.c_int, C.c_int,
                                    C.POINTER(C.c_uint)]),
        "qdc_lane_plan": (C.c_int, [C.c_uint, C.c_uint, C.c_uint, C.c_uint, C.c_int,
                                    C.POINTER(C.c_uint)]),
        "qdc_spec_selftest": (C.c_char_p, [C.c_uint, C.POINTER(C.c_uint), C.POINTER(C.c_uint),
                                           C.POINTER(C.c_uint), C.POINTER(C.c_ulonglong), _S,
                                           C.c_char_p, _S]),
        "qdc_jit_stats": (_S, [C.POINTER(C.c_double), _S]),
        "qdc_jit_wait": (_S, [C.c_double]),
        "qdc_check_schedule": (_E, [_S, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_uint),
                                    C.POINTER(C.c_uint), _S, C.POINTER(C.c_size_t),
                                    C.POINTER(C.c_size_t)]),
        "qdc_spec_selftest_batch": (C.c_char_p, [C.c_uint, C.POINTER(C.c_size_t), _S,
                                                 C.POINTER(C.c_uint), C.POINTER(C.c_uint),
                                                 C.POINTER(C.c_uint), C.POINTER(C.c_ulonglong),
                                                 C.c_char_p, _S]),
        "qdc_jit_dir": (_E, [C.c_char_p, _S]),
        "qdc_precompile": (_E, [_S, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_uint),
                                C.POINTER(C.c_uint), _S, _P, _P, _S, _P, _P, _S, _P, _P, _S,
                                C.POINTER(C.c_size_t)]),
        "qdc_trace_program": (_E, [_S, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_uint),
                                   C.POINTER(C.c_uint), _S, _P, _P, _S, _P, _P, _S, _P, _P, _S,
                                   _P, _S, C.POINTER(C.c_size_t)]),
        "qdc_spec_fingerprint": (_E, [C.c_char_p, C.c_char_p, C.c_char_p,
                                      C.POINTER(C.c_ulonglong), C.POINTER(C.c_ulonglong)]),
        "qdc_rq_plan": (_S, [C.c_uint, C.c_uint, C.POINTER(C.c_uint), C.POINTER(C.c_uint),
                             C.POINTER(C.c_uint), C.POINTER(C.c_ulonglong), _S,
                             C.POINTER(C.c_uint), _S]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_LIBS: dict = {}


def lib_path(precision: str) -> Path:
    """In-tree build; QDC_LIB_DIR selects another build of the same library (experiments)."""
    d = Path(os.environ["QDC_LIB_DIR"]) if os.environ.get("QDC_LIB_DIR") else LIB_DIR
    return d / f"libqdc_{precision}.so"


def load(precision: str = "f32"):
    """Load (once) the HIP library of the given precision.  Raises if it was not built."""
    if precision not in PRECISIONS:
        raise ValueError(f"precision must be one of {sorted(PRECISIONS)}, got {precision!r}")
    if precision not in _LIBS:
        path = lib_path(precision)
        if not path.exists():
            raise ImportError(
                f"HIP extension {path} is not built (run `python -c 'import __graft_entry__ as g;"
                f" g.build()'` or `make -C differentiable-quantum-circuit-cuda_amd/csrc`); "
                "there is no CPU fallback.")
        _LIBS[precision] = _proto(C.CDLL(str(path)))
    return _LIBS[precision]


def default_precision() -> str:
    p = os.environ.get("QDC_PRECISION", "f32").lower()
    return "f64" if p in ("f64", "double", "complex128") else "f32"


def check(err):
    if err:
        raise PanicException(err.decode() if isinstance(err, bytes) else str(err))


def ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)

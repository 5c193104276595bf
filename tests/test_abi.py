"""The C-ABI libraries (CPU only): they load, export every entry point include/qdc/*.h declares,
report their precision, and fail loudly — never fall back — when no GPU is present."""
import ctypes
import re
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
HEADERS = sorted((ROOT / "include" / "qdc").glob("*.h"))


def declared_functions():
    names = set()
    for h in HEADERS:
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b([a-z_][a-z0-9_]*)\s*\(", text, re.M):
            name = m.group(1)
            if name not in ("if", "for", "while", "return", "sizeof", "defined"):
                names.add(name)
    return names


def test_headers_declare_the_reference_abi():
    names = declared_functions()
    # the 18 functions of src/primitives_bind.rs:15-119
    ref = {"set2standard", "get_state", "drop_state", "copy_to_host", "q1gate", "q1gate_inv",
           "q2gate", "q2gate_inv", "q2gate_diag", "set_from_host", "get_q1density",
           "get_q2density", "q1grad", "q2grad", "q2grad_diag", "conj_and_double", "add", "copy"}
    assert ref <= names, ref - names


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_library_exports_every_declared_symbol(prec):
    from quantum_differentiable_circuit import _native
    path = _native.lib_path(prec)
    assert path.exists(), f"{path} not built"
    lib = ctypes.CDLL(str(path))
    missing = [n for n in sorted(declared_functions()) if not hasattr(lib, n)]
    assert not missing, missing
    lib.qdc_build_info.restype = ctypes.c_char_p
    assert lib.qdc_build_info().decode().startswith(f"qdc {prec}")


def test_python_binding_table_matches_headers():
    from quantum_differentiable_circuit import _native
    assert set(_native.PRIMITIVES) | set(_native.RUNTIME) == declared_functions()


def test_no_gpu_means_loud_failure():
    """Without a GPU the product path raises the HIP error; there is no CPU fallback."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    import quantum_differentiable_circuit as q
    with pytest.raises(q.PanicException, match="HIP ERROR"):
        q.circuit_class("f32")(4)
    with pytest.raises(q.PanicException, match="HIP ERROR"):
        q.QuantizedTensor.new_standard(4, "f64")


def test_missing_library_is_an_import_error(tmp_path, monkeypatch):
    from quantum_differentiable_circuit import _native
    monkeypatch.setattr(_native, "LIB_DIR", tmp_path)
    monkeypatch.setattr(_native, "_LIBS", {})
    with pytest.raises(ImportError, match="no CPU fallback"):
        _native.load("f32")


def test_oracle_is_not_imported_by_the_product():
    pkg = ROOT / "differentiable-quantum-circuit-cuda_amd"
    for f in list(pkg.rglob("*.py")) + list(pkg.rglob("*.hip")) + list(pkg.rglob("*.hpp")):
        text = f.read_text()
        assert "import oracle" not in text and "from oracle" not in text, f
        assert "cpu_ref" not in text and "cref" not in text, f


def test_flatten_helpers():
    import quantum_differentiable_circuit as q
    from quantum_differentiable_circuit import _flatten, _array1
    g = [np.arange(4, dtype=np.complex64), np.arange(16, dtype=np.complex64)]
    flat, lens = _flatten(g, np.complex64, "x", "m")
    assert flat.size == 20 and list(lens) == [4, 16]
    with pytest.raises(TypeError):
        _array1(np.zeros(4, np.complex128), np.dtype(np.complex64), "x")
    with pytest.raises(TypeError):
        _array1(np.zeros((2, 2), np.complex64), np.dtype(np.complex64), "x")
    with pytest.raises(q.PanicException, match="Gate is not contiguous."):
        _flatten([np.zeros(8, np.complex64)[::2]], np.complex64, "x", "Gate is not contiguous.")

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
    # the one-pass gate path: same result, same errors as _array1 + _flatten
    from quantum_differentiable_circuit import _flat_gates
    dt = np.dtype(np.complex64)
    flat2, lens2 = _flat_gates(g, dt, "x")
    assert np.array_equal(flat2, flat) and list(lens2) == [4, 16] and lens2.dtype == np.uintp
    with pytest.raises(TypeError, match="argument 'var_gates'"):
        _flat_gates(g + [np.zeros(4, np.complex128)], dt, "var_gates")
    with pytest.raises(TypeError):
        _flat_gates([[1, 2]], dt, "x")
    with pytest.raises(q.PanicException, match="Gate is not contiguous."):
        _flat_gates([np.zeros(8, np.complex64)[::2]], dt, "x")
    empty, elens = _flat_gates([], dt, "x")
    assert empty.size == 1 and elens.size == 1


# ------------------------------------------------------------------------------------------
# Rust views of the C ABI: the reference's primitives_bind.rs against primitives.h, and the
# circuit_bind.rs block of INTEGRATION.md §3a against circuit.h (names, arity, every type)
# ------------------------------------------------------------------------------------------
C_TO_RUST = {
    "void": None, "size_t": "usize", "int": "c_int", "unsigned": "c_uint", "double": "f64",
    "const char*": "*const c_char", "char*": "*mut c_char",
    "qdc_complex*": "*mut Complex", "const qdc_complex*": "*const Complex",
    "qdc_complex**": "*mut *mut Complex",
    "size_t*": "*mut usize", "const size_t*": "*const usize",
    "int*": "*mut c_int", "const int*": "*const c_int",
    "unsigned*": "*mut c_uint", "const unsigned*": "*const c_uint",
    "unsigned long long*": "*mut c_ulonglong", "const unsigned long long*": "*const c_ulonglong",
    "double*": "*mut f64", "const unsigned char*": "*const u8",
    "unsigned char[128]": "*mut u8", "const unsigned char[128]": "*const u8",
    "qdc_circuit*": "*mut QdcCircuit", "const qdc_circuit*": "*const QdcCircuit",
    "qdc_circuit**": "*mut *mut QdcCircuit", "qdc_comm*": "*mut QdcComm",
    "qdc_comm**": "*mut *mut QdcComm", "qdc_kernel_stat*": "*mut QdcKernelStat",
    "qdc_plan_op*": "*mut QdcPlanOp", "const qdc_plan_op*": "*const QdcPlanOp",
    "qdc_trace_op*": "*mut QdcTraceOp",
}


def c_declarations(header):
    """{name: (return type, [parameter types])} of a C header, types normalised"""
    text = re.sub(r"/\*.*?\*/", "", header.read_text(), flags=re.S)
    text = re.sub(r"#.*", "", text)
    text = re.sub(r"typedef struct[^;]*?\{.*?\}\s*\w+\s*;", "", text, flags=re.S)
    text = re.sub(r"enum\s+\w+\s*\{.*?\};", "", text, flags=re.S)

    def norm(t):
        t = " ".join(t.replace("*", " * ").split())
        return t.replace(" *", "*").replace("* ", "*") if "*" in t else t

    out = {}
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b([a-z_][a-z0-9_]*)\s*\(([^;{]*?)\)\s*;", text, re.S):
        ret, name, params = norm(m.group(1)), m.group(2), m.group(3).strip()
        types = []
        if params and params != "void":
            for p in params.split(","):
                p = " ".join(p.split())
                arr = re.search(r"\[(\d+)\]$", p)
                p = re.sub(r"\[\d+\]$", "", p)
                t = norm(re.sub(r"\b\w+$", "", p))  # drop the parameter name
                types.append(t + (f"[{arr.group(1)}]" if arr else ""))
        out[name] = (ret, types)
    return out


def rust_declarations(text):
    """{name: (return type or None, [parameter types])} of the fns in `extern "C"` blocks"""
    out = {}
    for block in re.findall(r'extern "C" \{(.*?)\n\}', text, re.S):
        block = re.sub(r"//.*", "", block)
        for m in re.finditer(r"fn\s+(\w+)\s*\((.*?)\)\s*(?:->\s*([^;]+))?;", block, re.S):
            name, params, ret = m.group(1), m.group(2), m.group(3)
            types = [" ".join(p.split(":", 1)[1].split()) for p in params.split(",") if p.strip()]
            out[name] = (" ".join(ret.split()) if ret else None, types)
    return out


def _compare(cdecl, rdecl, names):
    for name in sorted(names):
        cret, cparams = cdecl[name]
        rret, rparams = rdecl[name]
        assert C_TO_RUST[cret] == rret, (name, cret, rret)
        assert len(cparams) == len(rparams), (name, cparams, rparams)
        for i, (ct, rt) in enumerate(zip(cparams, rparams)):
            assert C_TO_RUST[ct] == rt, (name, i, ct, rt)


def test_integration_rust_block_matches_circuit_header():
    """INTEGRATION.md §3a declares every function of include/qdc/circuit.h for a Rust host, with
    the C types' Rust equivalents (the fused runtime's path from circuit.rs)."""
    cdecl = c_declarations(ROOT / "include" / "qdc" / "circuit.h")
    md = (ROOT / "INTEGRATION.md").read_text()
    blocks = [b for b in re.findall(r"```rust\n(.*?)```", md, re.S) if "qdc_circuit_new" in b and 'extern "C"' in b]
    assert len(blocks) == 1
    rdecl = rust_declarations(blocks[0])
    assert set(rdecl) == set(cdecl), (set(cdecl) ^ set(rdecl))
    _compare(cdecl, rdecl, cdecl)


REF_BIND = Path("/root/reference/src/primitives_bind.rs")


@pytest.mark.skipif(not REF_BIND.exists(), reason="reference tree not present")
def test_primitives_header_matches_reference_bindings():
    """include/qdc/primitives.h declares the 18 functions of src/primitives_bind.rs:15-119 with
    the types the reference's Rust binds them with (so its crate links libqdc unchanged)."""
    cdecl = c_declarations(ROOT / "include" / "qdc" / "primitives.h")
    rdecl = rust_declarations(REF_BIND.read_text().replace("pub(super) ", ""))
    assert len(rdecl) == 18 and set(rdecl) <= set(cdecl), set(rdecl) - set(cdecl)
    _compare(cdecl, rdecl, rdecl)

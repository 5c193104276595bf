"""Specialized reverse passes (csrc/qdc_spec.hpp, qdc_jit.hpp) on CPU: the runtime's source
generator and hipcc compile a pass program's straight-line kernel for gfx950 (the GPU box does
the same at a circuit's first call, then loads the code object).  Checks that the code object is
a gfx950 offload bundle, that one program maps to one kernel (the cache key), and that the
generated kernel keeps the interpreted kernel's resources (<= 256 VGPRs, 2 waves/SIMD) without
its per-stage register copies.  Parity on the GPU: tests/test_gpu_fusion.py."""
import os
import subprocess

import numpy as np
import pytest

from test_rq_plan import random_pass

pytestmark = pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")


@pytest.fixture(autouse=True)
def jit_dir(tmp_path, monkeypatch):
    monkeypatch.setenv("QDC_JIT_DIR", str(tmp_path))


def _passes(seed, count):
    rng = np.random.default_rng(seed)
    out = []
    for k in range(count):
        stages, deps = random_pass(rng, 11, int(rng.integers(6, 16)), brick=bool(k % 2))
        out.append((stages, deps))
    return out


def test_spec_kernel_compiles_for_gfx950_and_is_keyed_by_program():
    import quantum_differentiable_circuit as q
    (st1, d1), (st2, d2) = _passes(3, 2)
    name1, obj1 = q.spec_selftest(11, st1, d1)
    assert name1.startswith("qdc_spec_") and os.path.getsize(obj1) > 10000
    bundle = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o",
                             "--input=" + obj1], capture_output=True, text=True)
    assert "gfx950" in bundle.stdout, bundle.stdout + bundle.stderr
    # the same program again: the same kernel (no recompilation); another program: another one
    assert q.spec_selftest(11, st1, d1) == (name1, obj1)
    name2, _ = q.spec_selftest(11, st2, d2)
    assert name2 != name1


def test_spec_kernel_resources_and_no_stage_copies(tmp_path):
    import quantum_differentiable_circuit as q
    stages, deps = _passes(5, 1)[0]
    name, obj = q.spec_selftest(11, stages, deps)
    src = os.path.join(os.path.dirname(obj), name + "." + str(os.getpid()) + ".hip")
    assert os.path.exists(src)
    csrc = os.path.join(os.path.dirname(q.__file__), "..", "csrc")
    inc = os.path.join(csrc, "..", "..", "include")
    asm = tmp_path / "k.s"
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                        "-I" + inc, "-I" + csrc, "-S", "--cuda-device-only", "-o", str(asm), src],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    text = asm.read_text()
    body = text[text.index(name + ":"):text.index(".Lfunc_end0")]
    vgpr = int(text.split(".amdhsa_next_free_vgpr")[1].split()[0])
    assert vgpr <= 256
    # the interpreted kernel copies ~63 register pairs after every stage; straight-line code
    # keeps at most a handful of moves in total
    assert body.count("v_mov_b64") < 32, body.count("v_mov_b64")


def test_spec_forward_pass_kernel(tmp_path):
    """One-state forward passes (k_rq<false, 256, true> with the program inlined): a
    qdc_specf_ kernel, no scratch, within the generic kernel's 128 VGPRs."""
    import quantum_differentiable_circuit as q
    rng = np.random.default_rng(11)
    stages, deps = random_pass(rng, 12, 12, brick=False)
    name, obj = q.spec_selftest(12, stages, deps)
    assert name.startswith("qdc_specf_") and os.path.getsize(obj) > 10000
    src = os.path.join(os.path.dirname(obj), name + "." + str(os.getpid()) + ".hip")
    csrc = os.path.join(os.path.dirname(q.__file__), "..", "csrc")
    inc = os.path.join(csrc, "..", "..", "include")
    asm = tmp_path / "k.s"
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                        "-I" + inc, "-I" + csrc, "-S", "--cuda-device-only", "-o", str(asm), src],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    text = asm.read_text()
    meta = text[text.index(".amdhsa_kernel " + name):]
    assert int(meta.split(".amdhsa_next_free_vgpr")[1].split()[0]) <= 128
    assert int(meta.split(".amdhsa_private_segment_fixed_size")[1].split()[0]) == 0
    # a tile no specialized kernel runs: refused
    with pytest.raises(RuntimeError):
        q.spec_selftest(13, stages, deps)


@pytest.mark.parametrize("tile_bits,prefix", [(10, "qdc_spec_d_"), (11, "qdc_specf_d_")])
def test_spec_f64_pass_kernels(tmp_path, tile_bits, prefix):
    """f64 passes: two-state reverse (k_rw<true, 1, false, 1>, 2^10 tiles) and one-state
    (k_rw<false, 1, false, 2>, 2^11 tiles) written out per program, compiled with -DQDC_F64:
    no scratch, no per-stage copies, within 256 VGPRs."""
    import quantum_differentiable_circuit as q
    rng = np.random.default_rng(tile_bits)
    stages, deps = random_pass(rng, tile_bits, 10, brick=False)
    name, obj = q.spec_selftest(tile_bits, stages, deps, precision="f64")
    assert name.startswith(prefix) and os.path.getsize(obj) > 10000
    src = os.path.join(os.path.dirname(obj), name + "." + str(os.getpid()) + ".hip")
    csrc = os.path.join(os.path.dirname(q.__file__), "..", "csrc")
    inc = os.path.join(csrc, "..", "..", "include")
    asm = tmp_path / "k.s"
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-DQDC_F64",
                        "-I" + inc, "-I" + csrc, "-S", "--cuda-device-only", "-o", str(asm), src],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    text = asm.read_text()
    meta = text[text.index(".amdhsa_kernel " + name):]
    assert int(meta.split(".amdhsa_next_free_vgpr")[1].split()[0]) <= 256
    assert int(meta.split(".amdhsa_private_segment_fixed_size")[1].split()[0]) == 0
    body = text[text.index(name + ":"):]
    body = body[:body.index(".Lfunc_end")]
    assert body.count("v_mov_b64") < 32

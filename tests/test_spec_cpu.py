"""Specialized reverse passes (csrc/qdc_spec.hpp, qdc_jit.hpp) on CPU: the runtime's source
generator and hipcc compile a pass program's straight-line kernel for gfx950 (the GPU box does
the same at a circuit's first call, then loads the code object).  Checks that the code object is
a gfx950 offload bundle, that one program maps to one kernel (the cache key), and that the
generated kernel keeps the interpreted kernel's resources (<= 256 VGPRs, 2 waves/SIMD) without
its per-stage register copies.  The cache: kernel names carry the build fingerprint (-D
switches, compiler, header bytes), so an ablation build, a touched header or another compiler
never load another build's code object; objects are validated before use; the directory must
be private; and the processes of a job compile each kernel once.  Parity on the GPU:
tests/test_gpu_fusion.py."""
import json
import os
import shutil
import subprocess
import sys
import textwrap
from pathlib import Path

import numpy as np
import pytest

from test_rq_plan import random_pass

pytestmark = pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")


ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "differentiable-quantum-circuit-cuda_amd"
HDR = 40  # qdc_jit.hpp JitObjHeader in front of hipcc's output


@pytest.fixture(autouse=True)
def jit_dir(tmp_path, monkeypatch):
    monkeypatch.setenv("QDC_JIT_DIR", str(tmp_path))
    monkeypatch.setenv("QDC_JIT_KEEP", "1")  # the tests read the generated sources back


def _payload(obj, tmp_path):
    """hipcc's output inside a cached code object (behind the 40-byte header)"""
    raw = Path(obj).read_bytes()
    assert raw[:8] == b"QDCJIT2\0", raw[:8]
    out = tmp_path / "payload.hsaco"
    out.write_bytes(raw[HDR:])
    return str(out)


def _run(code, env=None, timeout=300):
    """a fresh process (its own SpecJit state) running `code`; returns its last stdout line as JSON"""
    e = dict(os.environ)
    e.update(env or {})
    pre = (f"import sys, json; sys.path[:0] = [{str(ROOT)!r}, {str(PKG)!r}, {str(ROOT / 'tests')!r}]\n")
    r = subprocess.run([sys.executable, "-c", pre + textwrap.dedent(code)], env=e,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout + r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1]), r.stderr


def _passes(seed, count):
    rng = np.random.default_rng(seed)
    out = []
    for k in range(count):
        stages, deps = random_pass(rng, 11, int(rng.integers(6, 16)), brick=bool(k % 2))
        out.append((stages, deps))
    return out


def test_spec_kernel_compiles_for_gfx950_and_is_keyed_by_program(tmp_path):
    import quantum_differentiable_circuit as q
    (st1, d1), (st2, d2) = _passes(3, 2)
    name1, obj1 = q.spec_selftest(11, st1, d1)
    assert name1.startswith("qdc_spec_") and os.path.getsize(obj1) > 10000
    bundle = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o",
                             "--input=" + _payload(obj1, tmp_path)], capture_output=True, text=True)
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


# ------------------------------------------------------------------------------------------
# the cache: build fingerprint, validated objects, private directory, one compile per kernel
# ------------------------------------------------------------------------------------------
def _copy_tree(tmp_path):
    """csrc + include as they sit next to the library (csrc/../../include)"""
    dst = tmp_path / "tree"
    shutil.copytree(PKG / "csrc", dst / "pkg" / "csrc")
    shutil.copytree(ROOT / "include", dst / "include")
    return dst / "pkg" / "csrc"


def test_fingerprint_covers_defines_compiler_and_headers(tmp_path):
    """The kernel-name fingerprint changes with any -D switch the library was built with
    (QDC_RQ_ABL: a timing-only build), the compiler identity, and any byte of a kernel header;
    the header hash equals the one the Makefile compiles in (csrc/src_fp.py)."""
    import quantum_differentiable_circuit as q
    r = subprocess.run([sys.executable, str(PKG / "csrc" / "src_fp.py"), str(PKG / "csrc"),
                        str(ROOT / "include")], capture_output=True, text=True, check=True)
    assert int(r.stdout, 16) == q.spec_fingerprint(PKG / "csrc", "x")[1]
    csrc = _copy_tree(tmp_path)
    own, sh = q.spec_fingerprint(csrc, "hipcc A")  # this library's own -D switches
    assert q.spec_fingerprint(csrc, "hipcc A") == (own, sh)
    defs = ("-DQDC_DYN_TAIL=1 -DQDC_FMAX_OPS=40 -DQDC_FMAX_GRAD_RQ=16 -DQDC_RQ_PF_WAVES=2 "
            "-DQDC_RW_WAVES=2 -DQDC_RW_WAVES_ONE=2 -DQDC_RQ_ABL=0 -DQDC_RQ_GSPLIT=0")
    abl = defs.replace("QDC_RQ_ABL=0", "QDC_RQ_ABL=1")
    assert q.spec_fingerprint(csrc, "hipcc A", defines=defs)[0] != \
        q.spec_fingerprint(csrc, "hipcc A", defines=abl)[0]
    assert q.spec_fingerprint(csrc, "hipcc B")[0] != own
    hdr = csrc / "qdc_rq.hpp"
    hdr.write_text(hdr.read_text() + "\n// touched\n")
    fp2, sh2 = q.spec_fingerprint(csrc, "hipcc A")
    assert sh2 != sh and fp2 != own
    inc = csrc.parent.parent / "include" / "qdc" / "circuit.h"
    inc.write_text(inc.read_text() + "\n")
    assert q.spec_fingerprint(csrc, "hipcc A")[1] not in (sh, sh2)


ABL_LIB = PKG / "lib-abl" / "libqdc_f32.so"


@pytest.mark.skipif(not ABL_LIB.exists(), reason="ablation build (make -C csrc abl) not built")
def test_ablation_build_never_shares_kernels(tmp_path):
    """Two builds that differ only in -DQDC_RQ_ABL (the production library and the timing-only
    ablation library, csrc/Makefile `abl`) compile the same pass program into differently named
    code objects in one QDC_JIT_DIR, so neither ever loads the other's kernels."""
    (stages, deps), = _passes(7, 1)
    out = {}
    for tag, libdir in (("abl", ABL_LIB.parent), ("prod", PKG / "lib")):
        out[tag], _ = _run(f"""
            import quantum_differentiable_circuit as q
            name, obj = q.spec_selftest(11, {stages!r}, {deps!r})
            print(json.dumps([name, obj, q.jit_stats('f32')['compiled'], q.jit_dir('f32')]))
            """, {"QDC_LIB_DIR": str(libdir)})
    (na, oa, ca, da), (np_, op, cp, dp) = out["abl"], out["prod"]
    assert da == dp == str(tmp_path)
    assert na != np_ and oa != op and os.path.exists(oa) and os.path.exists(op)
    assert ca == 1 and cp == 1  # the production process compiled its own kernel


def test_stale_and_corrupt_code_objects_are_rebuilt(tmp_path):
    """A cached object whose header names another build, or whose bytes are cut short, is never
    loaded: the next process compiles the kernel again."""
    (stages, deps), = _passes(8, 1)
    code = f"""
        import quantum_differentiable_circuit as q
        name, obj = q.spec_selftest(11, {stages!r}, {deps!r})
        print(json.dumps([name, obj, q.jit_stats('f32')['compiled']]))
        """
    (name, obj, c1), _ = _run(code)
    assert c1 == 1
    (_, _, c2), _ = _run(code)
    assert c2 == 0  # valid: reused
    raw = bytearray(Path(obj).read_bytes())
    raw[8] ^= 0xFF  # the fingerprint of another build
    Path(obj).write_bytes(bytes(raw))
    (_, _, c3), _ = _run(code)
    assert c3 == 1
    Path(obj).write_bytes(Path(obj).read_bytes()[:-100])  # truncated
    (_, _, c4), _ = _run(code)
    assert c4 == 1
    assert Path(obj).read_bytes()[:8] == b"QDCJIT2\0"
    # good compiles leave no sources or logs behind (QDC_JIT_KEEP unset)
    _run(code, {"QDC_JIT_KEEP": "0", "QDC_JIT_DIR": str(tmp_path / "clean")})
    left = sorted(p.name for p in (tmp_path / "clean").iterdir())
    assert all(p.endswith((".qco", ".lock")) for p in left), left


def test_cache_directory_must_be_private(tmp_path):
    """QDC_JIT_DIR writable by others, or a symlink, turns specialization off (another user could
    plant code objects); the default is a 0700 directory under $HOME/.cache."""
    code = """
        import quantum_differentiable_circuit as q
        try:
            d = q.jit_dir('f32')
        except RuntimeError as e:
            d = 'off: ' + str(e)
        print(json.dumps(d))
        """
    open_dir = tmp_path / "open"
    open_dir.mkdir()
    open_dir.chmod(0o777)
    d, err = _run(code, {"QDC_JIT_DIR": str(open_dir)})
    assert d.startswith("off") and "writable by other users" in err
    real = tmp_path / "real"
    real.mkdir(mode=0o700)
    link = tmp_path / "link"
    link.symlink_to(real)
    d, err = _run(code, {"QDC_JIT_DIR": str(link)})
    assert d.startswith("off") and "not a directory" in err
    home = tmp_path / "home"
    home.mkdir(mode=0o700)
    env = {"HOME": str(home), "XDG_CACHE_HOME": ""}
    e = dict(os.environ)
    e.pop("QDC_JIT_DIR", None)
    os.environ.pop("QDC_JIT_DIR", None)
    try:
        d, _ = _run(code, env)
    finally:
        os.environ["QDC_JIT_DIR"] = str(tmp_path)
    assert d == str(home / ".cache" / "qdc_jit")
    assert (os.stat(d).st_mode & 0o777) == 0o700


def test_touched_headers_turn_specialization_off(tmp_path):
    """Kernel headers that are not the ones the library was built from (QDC_SRC_FP) would
    compile kernels that disagree with the library's host code: specialization turns off."""
    csrc = _copy_tree(tmp_path)
    hdr = csrc / "qdc_spec.hpp"
    hdr.write_text(hdr.read_text() + "\n// touched\n")
    (stages, deps), = _passes(9, 1)
    d, err = _run(f"""
        import quantum_differentiable_circuit as q
        try:
            q.spec_selftest(11, {stages!r}, {deps!r})
            print(json.dumps("compiled"))
        except RuntimeError as e:
            print(json.dumps("off: " + str(e)))
        """, {"QDC_SRC_DIR": str(csrc)})
    assert d.startswith("off") and "not the ones this library was built from" in err


def test_processes_of_a_job_compile_each_kernel_once(tmp_path):
    """Four processes sharing one cache directory (the ranks of a multi-process job, two hipcc
    processes each) ask for the same eight kernels at the same moment: every kernel is compiled
    by exactly one of them (per-kernel locks, taken a compile batch at a time, so the processes
    share the work), the others wait for it and use its code object."""
    progs = _passes(10, 8)
    go = tmp_path / "go"
    code = f"""
        import os, time
        import quantum_differentiable_circuit as q
        while not os.path.exists({str(go)!r}):
            time.sleep(0.01)
        names = q.spec_selftest_batch(11, {[(s, d) for s, d in progs]!r})
        s = q.jit_stats('f32')
        print(json.dumps([names, s['compiled'], s['waited']]))
        """
    e = dict(os.environ, QDC_JIT_KEEP="0", QDC_JIT_JOBS="2")
    pre = (f"import sys, json; sys.path[:0] = [{str(ROOT)!r}, {str(PKG)!r}]\n")
    procs = [subprocess.Popen([sys.executable, "-c", pre + textwrap.dedent(code)], env=e,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for _ in range(4)]
    import time
    time.sleep(1.5)  # every process imported and is polling
    go.write_text("")
    res = []
    for p in procs:
        out, err = p.communicate(timeout=600)
        assert p.returncode == 0, out + err
        res.append(json.loads(out.strip().splitlines()[-1]))
    names = {tuple(r[0]) for r in res}
    assert len(names) == 1 and len(set(next(iter(names)))) == 8
    assert sum(r[1] for r in res) == 8, res  # each kernel compiled once in the whole job
    assert sum(1 for r in res if r[1] > 0) >= 2, res  # by more than one process
    assert sum(r[2] for r in res) >= 1, res  # and someone waited for another's compile


@pytest.mark.parametrize("pf", [0, 0x200])
def test_spec_one_wave_forward_pass_kernel(tmp_path, pf):
    """One-state passes on 2^11 tiles (QDC_TILE1_CHUNKS=1024 with QDC_RW bit 1: k_rw<false, 2,
    false, 1, true>, one wave, five register slots; with QDC_RW bit 3 the next tile prefetched
    into pinned VGPRs, k_rw<false, 2, true, 1, true>) written out per program: no scratch,
    within the two waves per SIMD the generic kernel runs at."""
    import quantum_differentiable_circuit as q
    rng = np.random.default_rng(21)
    stages, deps = random_pass(rng, 11, 12, brick=True)
    name, obj = q.spec_selftest(11 | 0x100 | 0x400 | pf, stages, deps)  # (full buffer)
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
    assert int(meta.split(".amdhsa_next_free_vgpr")[1].split()[0]) <= 256
    assert int(meta.split(".amdhsa_private_segment_fixed_size")[1].split()[0]) == 0


@pytest.mark.parametrize("tile_bits,prefix", [(11 | 0x100, "qdc_specf_"), (11, "qdc_spec_")])
def test_spec_half_buffer_relayouts(tmp_path, tile_bits, prefix):
    """One-wave five-slot programs (one-state 2^11 tiles and the two-state reverse passes) plan
    every relayout to keep a register slot in place (rq_plan keep) and exchange through half the
    LDS buffer in two rounds (spec_xchg_half): 8 KiB (one-state) / 10 KiB (two-state, with the
    Gamma accumulators) of LDS per wave instead of 16 / 18.  | 0x400 keeps the full buffer
    (another kernel)."""
    import quantum_differentiable_circuit as q
    rng = np.random.default_rng(23)
    stages, deps = random_pass(rng, 11, 14, brick=True)
    name, obj = q.spec_selftest(tile_bits, stages, deps)
    full, _ = q.spec_selftest(tile_bits | 0x400, stages, deps)
    assert name.startswith(prefix) and full.startswith(prefix) and name != full
    src = os.path.join(os.path.dirname(obj), name + "." + str(os.getpid()) + ".hip")
    assert "spec_xchg_half<" in open(src).read() and "Prog, true>" in open(src).read()
    csrc = os.path.join(os.path.dirname(q.__file__), "..", "csrc")
    inc = os.path.join(csrc, "..", "..", "include")
    asm = tmp_path / "k.s"
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                        "-I" + inc, "-I" + csrc, "-S", "--cuda-device-only", "-o", str(asm), src],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    text = asm.read_text()
    meta = text[text.index(".amdhsa_kernel " + name):]
    lds = int(meta.split(".amdhsa_group_segment_fixed_size")[1].split()[0])
    assert lds == (8192 if tile_bits & 0x100 else 10240), lds
    # the one-state kind is compiled for 5 waves per SIMD (<= 102 VGPRs): a few registers of
    # the relayout addressing spill (~50 B per lane, measured faster than 4 waves without)
    scratch = int(meta.split(".amdhsa_private_segment_fixed_size")[1].split()[0])
    vgpr = int(meta.split(".amdhsa_next_free_vgpr")[1].split()[0])
    if tile_bits & 0x100:
        assert scratch <= 128 and vgpr <= 102, (scratch, vgpr)
    else:
        assert scratch == 0, scratch

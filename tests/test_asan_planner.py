"""The host planners (qdc_shard.hpp remap planner, qdc_fusion.hpp pass scheduler and register
layout planner, qdc_stage.hpp, qdc_device.hpp plan_gate) under AddressSanitizer + UndefinedBehaviorSanitizer: the CPU
planner tests run in a child process against lib-asan/libqdc_{f32,f64}.so (make -C
differentiable-quantum-circuit-cuda_amd/csrc asan; built by __graft_entry__.build()) with the
ASan runtime preloaded.  Any sanitizer report aborts the child (abort_on_error, halt_on_error)."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
ASAN_LIB = ROOT / "differentiable-quantum-circuit-cuda_amd" / "lib-asan"
RT = Path("/opt/rocm/lib/llvm/lib/clang/22/lib/linux/libclang_rt.asan-x86_64.so")


def test_planners_under_asan_ubsan():
    if not (ASAN_LIB / "libqdc_f32.so").exists() or not (ASAN_LIB / "libqdc_f64.so").exists():
        pytest.skip("ASan build absent (make -C differentiable-quantum-circuit-cuda_amd/csrc asan)")
    if not RT.exists():
        pytest.skip("clang ASan runtime not found")
    env = dict(os.environ, LD_PRELOAD=str(RT), QDC_LIB_DIR=str(ASAN_LIB),
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        "-m", "not gpu", "tests/test_fusion_schedule.py", "tests/test_rq_plan.py",
                        "tests/test_sharded_cpu.py", "tests/test_gate_plan.py"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert "ERROR: AddressSanitizer" not in tail and "runtime error:" not in tail, tail

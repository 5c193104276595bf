#!/usr/bin/env python3
"""Turn a rocprofv3 round (tools/gpu_round.sh output) into the committed profile artifacts.

HBM bytes per launch = FETCH_SIZE x 2 x 1024 + WRITE_SIZE x 1024, following
/opt/skills/guides/MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are KiB, and on gfx950
FETCH_SIZE reports exactly half the bytes of a wide (16 B/lane) coalesced streaming read —
every load of these kernels is a 16-byte nontemporal global_load_dwordx4 — so it is doubled.
FETCH_SIZE and WRITE_SIZE come from separate --pmc passes.

usage: python tools/pmc_summary.py gpurun_out/<tag> profiles/<round> [--prefix P] [--detail-only]
  --prefix P: the pass directories are P + pmc_FETCH_SIZE etc. (tools/gpu_f64.sh: f64_)
  --detail-only: write <round>_pmc_traffic.json only (not the f32 pmc_traffic.json bench reads)
"""
import csv
import hashlib
import json
import re
import shutil
import sys
from collections import defaultdict
from pathlib import Path

OPS = {0: "apply", 1: "reverse", 2: "reverse", 3: "inject", 4: "inject", 5: "density", 6: "grad"}
DIAG = {0: "apply_q2_diag", 1: "reverse_q2_diag", 2: "reverse_q2_diag", 3: "grad_q2_diag"}


def bench_name(kernel):
    """Map a HIP kernel symbol to the kernel names bench.py reports."""
    m = re.search(r"k_(direct|tile)<(\d+), (\d+)", kernel)
    if m:
        op, r = int(m.group(2)), int(m.group(3))
        return f"{OPS[op]}_q{1 if r == 2 else 2}"
    m = re.search(r"k_diag<(\d+)", kernel)
    if m:
        return DIAG[int(m.group(1))]
    m = re.search(r"k_fused<(true|false), \d+, (true|false), (true|false)(?:, \d+)?>", kernel)
    if m:  # <TWO, TB, HASRED, WF> -> the bench's per-variant names
        two, wf = m.group(1) == "true", m.group(3) == "true"
        return ("fused_reverse" if wf else "fused_inject") if two else \
               ("fused_apply" if wf else "fused_density")
    if kernel.startswith("qdc_spec_"):  # a specialized reverse pass (csrc/qdc_spec.hpp)
        return "fused_reverse"
    if kernel.startswith("qdc_specf_"):  # a specialized one-state forward pass
        return "fused_apply"
    m = re.search(r"k_r[qw]<(true|false), \d+[^>]*>", kernel)
    if m:  # register-resident gate passes (qdc_rq.hpp): k_rq<TWO, NT, PF>, k_rw<TWO, NE, PF>
        return "fused_reverse" if m.group(1) == "true" else "fused_apply"
    if "k_dens1<" in kernel:  # read-only one-qubit density passes (round 6)
        return "fused_density"
    if "k_elementwise<0>" in kernel:
        return "copy"
    if "k_elementwise<4>" in kernel:
        return "zero"
    if "k_finalize" in kernel:
        return "finalize"
    if "k_diag_inject" in kernel:
        return "inject_diag"
    if "k_dsum" in kernel:
        return "dsum"
    return None


def per_launch(path, counter):
    sums, counts = defaultdict(float), defaultdict(int)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = bench_name(r["Kernel_Name"])
        if name:
            sums[name] += float(r["Counter_Value"])
            counts[name] += 1
    return {k: sums[k] / counts[k] for k in sums}, dict(counts)


LIB = Path(__file__).resolve().parent.parent / "differentiable-quantum-circuit-cuda_amd" / "lib"


def lib_sha16(precision="f32"):
    """Identity of the library the counters were collected on (bench.py reports the traffic only
    for this same build, so a stale profile cannot be quoted after a kernel change)."""
    return hashlib.sha256((LIB / f"libqdc_{precision}.so").read_bytes()).hexdigest()[:16]


def main(src, dst, prefix="", detail_only=False):
    src, dst = Path(src), Path(dst)
    dst.parent.mkdir(parents=True, exist_ok=True)
    fetch, nf = per_launch(src / f"{prefix}pmc_FETCH_SIZE" / "pmc_counter_collection.csv", "FETCH_SIZE")
    write, nw = per_launch(src / f"{prefix}pmc_WRITE_SIZE" / "pmc_counter_collection.csv", "WRITE_SIZE")
    traffic = {}
    for k in sorted(set(fetch) | set(write)):
        traffic[k] = round(fetch.get(k, 0.0) * 2 * 1024 + write.get(k, 0.0) * 1024)
    detail = {k: {"FETCH_SIZE_KiB": fetch.get(k), "WRITE_SIZE_KiB": write.get(k),
                  "launches_fetch_pass": nf.get(k), "launches_write_pass": nw.get(k),
                  "hbm_bytes_per_launch": traffic[k]} for k in traffic}
    (dst.parent / f"{dst.name}_pmc_traffic.json").write_text(json.dumps(detail, indent=1) + "\n")
    if detail_only:
        print(json.dumps(detail, indent=1))
        return
    traffic["lib_sha16"] = lib_sha16()
    (dst.parent / "pmc_traffic.json").write_text(json.dumps(traffic, indent=1) + "\n")
    stats = src / "trace" / "trace_kernel_stats.csv"
    if stats.exists():
        shutil.copy(stats, dst.parent / f"{dst.name}_kernel_stats.csv")
    bench = src / "bench.log"
    if bench.exists():
        lines = [l for l in bench.read_text().splitlines() if l.startswith("{")]
        if lines:
            (dst.parent / f"{dst.name}_bench.json").write_text(lines[-1] + "\n")
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    a = sys.argv[1:]
    pre = a[a.index("--prefix") + 1] if "--prefix" in a else ""
    main(a[0], a[1], pre, "--detail-only" in a)

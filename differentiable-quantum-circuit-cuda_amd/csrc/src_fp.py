#!/usr/bin/env python3
"""Build-time hash of the kernel headers (QDC_SRC_FP): every csrc/*.hpp and include/qdc/*.h,
as (relative path, NUL, bytes, NUL) in sorted path order, FNV-1a 64 — the same bytes
qdc_jit.hpp spec_source_fp() hashes at run time, so a library can tell that the headers its
specialized kernels would compile against changed since it was built.

usage: src_fp.py CSRC_DIR INCLUDE_DIR  ->  prints 0x<16 hex digits>"""
import sys
from pathlib import Path


def fnv(h, data):
    for c in data:
        h = ((h ^ c) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def source_fp(csrc, inc):
    files = [("csrc/" + p.name, p) for p in Path(csrc).iterdir()
             if p.name.endswith(".hpp") and not p.name.startswith(".")]
    files += [("include/qdc/" + p.name, p) for p in (Path(inc) / "qdc").iterdir()
              if p.name.endswith(".h") and not p.name.startswith(".")]
    h = 1469598103934665603
    for rel, p in sorted(files, key=lambda f: f[0].encode()):
        h = fnv(h, rel.encode() + b"\0")
        h = fnv(h, p.read_bytes())
        h = fnv(h, b"\0")
    return h


if __name__ == "__main__":
    print(f"0x{source_fp(sys.argv[1], sys.argv[2]):016x}")

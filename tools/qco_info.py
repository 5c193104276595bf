#!/usr/bin/env python3
"""Resource usage of specialized-kernel code objects (qdc_jit.hpp .qco files: a 40-byte header,
then the gfx950 ELF): VGPRs, AGPRs, SGPRs, LDS, scratch and waves/SIMD, from the AMDHSA
metadata note (llvm-readelf --notes)."""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
BUNDLER = "/opt/rocm/lib/llvm/bin/clang-offload-bundler"


def info(path):
    raw = Path(path).read_bytes()[40:]
    with tempfile.TemporaryDirectory() as d:
        b, e = Path(d) / "k.bundle", Path(d) / "k.elf"
        b.write_bytes(raw)
        if raw.startswith(b"__CLANG_OFFLOAD_BUNDLE__"):  # hipcc --genco output
            subprocess.run([BUNDLER, "--unbundle", "--type=o", f"--input={b}", f"--output={e}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"], check=True)
        else:
            e.write_bytes(raw)
        out = subprocess.run([READELF, "--notes", str(e)], capture_output=True, text=True).stdout
    def get(key):
        m = re.search(r"\.%s:\s+(\d+)" % re.escape(key), out)
        return int(m.group(1)) if m else None
    return {"vgpr": get("vgpr_count"), "agpr": get("agpr_count"), "sgpr": get("sgpr_count"),
            "lds": get("group_segment_fixed_size"), "scratch": get("private_segment_fixed_size"),
            "vgpr_spill": get("vgpr_spill_count")}


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(Path(p).name, info(p))

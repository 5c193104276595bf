#!/usr/bin/env python3
"""Per-kernel summary of a dense k-qubit counter session (tools/r4_qk.sh: FETCH_SIZE,
WRITE_SIZE and SQ passes of tools/qk_once.py, rocprofv3 counter_collection CSVs): launches, HBM
bytes per launch against the algorithmic 2S (FETCH_SIZE x 2 x 1024 + WRITE_SIZE x 1024, the
gfx950 corrections of tools/pmc_summary.py) and the matrix cores' busy share
(SQ_VALU_MFMA_BUSY_CYCLES per SIMD, 256 CUs x 4 SIMDs, over GRBM_GUI_ACTIVE per XCD: the
counter comes summed over the 8 XCDs).
usage: qk_pmc_summary.py <fetch.csv> <write.csv> <sq.csv> [n=28] [bytes per amplitude=8]"""
import csv
import re
import sys
from collections import defaultdict

SIMDS = 256 * 4
XCDS = 8


def short(name):
    m = re.search(r"qdc::(k_qkl?)<(\d+), (\d+)(?:, (\d+))?(?:, (true|false))?>", name)
    return m.group(0) if m else None


def load(path):
    out = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        if k:
            out[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def main(fetch, write, sq, n=28, amp=8):
    algo = 2.0 * (1 << n) * amp
    f, w, s = load(fetch), load(write), load(sq)
    print("kernel,launches,hbm_bytes_per_launch,x_algorithmic_2S,mfma_busy_share")
    for k in sorted(set(f) | set(w) | set(s)):
        fe = f[k].get("FETCH_SIZE", [])
        wr = w[k].get("WRITE_SIZE", [])
        nl = max(len(fe), len(wr))
        b = (sum(fe) * 2 * 1024 / max(len(fe), 1)) + (sum(wr) * 1024 / max(len(wr), 1))
        mf, gr = s[k].get("SQ_VALU_MFMA_BUSY_CYCLES", []), s[k].get("GRBM_GUI_ACTIVE", [])
        busy = (sum(mf) / SIMDS) / (sum(gr) / XCDS) if mf and gr and sum(gr) else float("nan")
        print(f"{k},{nl},{b:.4g},{b / algo:.3f},{busy:.3f}")


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], a[1], a[2], *(int(x) for x in a[3:]))

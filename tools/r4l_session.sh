#!/bin/bash
# Single-gate tile defaults (far targets of one-state and reverse ops on 64 KiB tiles): the GPU
# suite, then the bench's whole single-gate sweep (every q1 position, 8 q2 pairs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4l}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  --deselect tests/test_gpu_drift.py::test_c5_full_size_10k_gates > "$OUT/tests.log" 2>&1
rc=$?; tail -2 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
grep -c "passes-by ATOL" "$OUT/tests.log"
timeout -k 10 900 python3 -u tools/micro_tune.py --reps 1 --q1 $(seq -s, 0 27) --q2 0:1,1:0,5:20,26:27,27:0,1:2,3:9,14:13 \
  --cfgs "-" --out "$OUT/sweep.json" > "$OUT/sweep.log" 2>&1 || exit $?
python3 - "$OUT/sweep.json" <<'PY'
import json, sys
t = [r for r in json.load(open(sys.argv[1])) if r["kernel"].startswith(("apply_", "reverse_"))]
w = min(t, key=lambda r: r["frac"])
print("cells", len(t), "below 70 %:", [(r["case"], r["kernel"], r["frac"]) for r in t if r["frac"] < 0.70], "min", w)
PY

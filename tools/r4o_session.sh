#!/bin/bash
# The n = 33 C5 test (three 64 GiB states, 10k gates, mirrored sweeps by default) and the CPU
# baseline's whole 20-layer C2 step at n = 28 (--cpu-layers 20: the reference's algorithm end to
# end on the box's cores, ~2.5 min).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4o}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_drift.py -v -s --timeout 800 --timeout-method thread \
  -k c5_full_size > "$OUT/c5_full.log" 2>&1
rc=$?; grep -E "drift|fd|passed|failed" "$OUT/c5_full.log" | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py --steps 1 --warmup 1 --cpu-layers 20 --no-gate-sample > "$OUT/cpu_full.log" 2> "$OUT/cpu_full.err" || exit $?
python3 -c "
import json
d = json.loads([l for l in open('$OUT/cpu_full.log') if l.startswith('{')][-1])
print(json.dumps(d['cpu_baseline'])[:1500])"

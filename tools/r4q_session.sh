#!/bin/bash
# The half-LDS occupancy probe (tools/r4p_session.sh), then the CPU baseline's whole 20-layer C2
# step at n = 28 (--cpu-layers 20), with a heartbeat file while the long host call runs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r4q}
mkdir -p "$OUT"
export TMPDIR=/tmp
TAG=${TAG:-r4q}/probe bash tools/r4p_session.sh || exit $?
(while sleep 30; do date >> "$OUT/heartbeat"; done) &
HB=$!
timeout -k 10 900 python -u bench.py --steps 1 --warmup 1 --cpu-layers 20 --no-gate-sample > "$OUT/cpu_full.log" 2> "$OUT/cpu_full.err"
rc=$?
kill $HB
[ $rc -eq 0 ] || exit $rc
python3 -c "
import json
d = json.loads([l for l in open('$OUT/cpu_full.log') if l.startswith('{')][-1])
print(json.dumps(d['cpu_baseline'])[:1500])"

#!/bin/bash
# Wider fused tile rows with matching permutation width: parity of the permuting passes under
# each setting, then a same-box A/B of the C2 bench (interleaved, REPS rounds).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TAG=${TAG:-lc_ab}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fusion.py -k permuting -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
CFGS="${CFGS:-- QDC_FUSE_LCMIN=4,QDC_RQ_PERM_LOW=5 QDC_FUSE_LCMIN=5,QDC_RQ_PERM_LOW=6 QDC_FUSE_LCMIN=4}" REPS=${REPS:-2} bash tools/ab_env.sh

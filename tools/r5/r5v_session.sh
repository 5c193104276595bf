#!/bin/bash
# Round 5v: dense k-qubit gate variants (QDC_QKL_VAR 1: pipelined, 3: half tiles at k = 5 not
# pipelined, 4 waves per SIMD), bench.py's dense sample at n = 28, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for v in 1 3 2 0 1 3; do
  echo "QDC_QKL_VAR=$v"
  QDC_QKL_VAR=$v timeout -k 10 120 python tools/r5/qk_sample.py || exit $?
done

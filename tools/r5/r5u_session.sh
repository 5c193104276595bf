#!/bin/bash
# Round 5u: the shard rehearsal with the final library (local shards / shard streams on one GPU,
# C2 n = 28).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
TAG=r5u STEPS_N=3 bash tools/shard_rehearsal.sh

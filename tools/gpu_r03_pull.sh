#!/bin/bash
# Pull placement re-checked on the current step: kernel pull (default), copy
# engine, capped pull grids.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r03pull
mkdir -p "$OUT"; cd "$ROOT"
ROUNDS=3 bash tools/ab_env_n.sh "GS_X=0" "GS_PULL_COPY=1" "GS_PULL_BLOCKS=16" "GS_PULL_BLOCKS=64" > "$OUT/ab.txt" 2>&1 || exit $?
tail -5 "$OUT/ab.txt"

#!/bin/bash
# Round-5 pass E: layer-1 forward K-chunk prefetch depth (GS_FWD_AHEAD 2 / 3 / 4), three alternating rounds.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r05e
mkdir -p "$OUT"; cd "$ROOT"
ROUNDS=3 timeout -k 10 1000 bash tools/ab_multi.sh graphsage-pytorch_amd/libgraphsage_amd.so graphsage-pytorch_amd/libgraphsage_amd_fa3.so graphsage-pytorch_amd/libgraphsage_amd_fa4.so > "$OUT/ab.txt" 2>&1; rc=$?
cat "$OUT/ab.txt"; exit $rc

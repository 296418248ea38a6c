#!/bin/bash
# Round-5 pass D: top-launch lab (v2 with the head fixes), then three
# alternating rounds of the bench on the new build (main) and the pruned
# round-start build (alt: graphsage-pytorch_amd/libgraphsage_amd_alt.so).
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r05d
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 120 tools/bin/top_lab tids > "$OUT/top_lab.txt" 2>&1; rc=$?
cat "$OUT/top_lab.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 bash tools/ab_so.sh > "$OUT/ab_so.txt" 2>&1; rc=$?
cat "$OUT/ab_so.txt"
exit $rc

#!/bin/bash
# Round-4 pass AE: top launch lab, the E GEMM on 8 waves (one tile per wave,
# -DGS_TOP_E8=1) against the default 4 waves (two tiles per wave).
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04ae
mkdir -p "$OUT"; cd "$ROOT"
for i in 1 2; do
  for V in base e8; do
    for M in plain tids; do
      echo "== $V $M round $i" >> "$OUT/top_lab_ab.txt"
      timeout -k 10 60 tools/bin/top_lab_$V $M >> "$OUT/top_lab_ab.txt" 2>&1 || exit $?
    done
  done
done
grep -E "==|per launch|hash|stage" "$OUT/top_lab_ab.txt"

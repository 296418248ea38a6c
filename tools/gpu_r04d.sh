#!/bin/bash
# Round-4 pass D: the top launch's W2 placement A/B in the lab (GS_TOP_WREG
# 0 = W2 in LDS for both GEMMs, 1 = E's operands in registers, 2 = both in
# registers, no LDS copy), three alternating rounds; outputs must hash equal.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04d
mkdir -p "$OUT"; cd "$ROOT"
for r in 1 2 3; do
  for m in 0 1 2; do
    echo "== WREG=$m round $r" >> "$OUT/top_lab.txt"
    GS_TOP_WREG=$m timeout -k 10 60 tools/bin/top_lab >> "$OUT/top_lab.txt" 2>&1 || exit $?
  done
done
grep -E "==|per launch|hash|stage" "$OUT/top_lab.txt"

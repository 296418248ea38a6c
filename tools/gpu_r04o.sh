#!/bin/bash
# Round-4 pass O: the top launch's dIn chain with every operand preloaded
# (GS_TOP_DIN_PRELOAD, lab A/B; outputs must hash equal).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04o
mkdir -p "$OUT"; cd "$ROOT"
for i in 1 2 3; do
  for V in 0 1; do
    echo "== din$V round $i" >> "$OUT/top_lab_din.txt"
    timeout -k 10 60 tools/bin/top_lab_din$V tids >> "$OUT/top_lab_din.txt" 2>&1 || exit $?
  done
done
grep -E "==|top kernel|hash|stage 6" "$OUT/top_lab_din.txt"

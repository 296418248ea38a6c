#!/bin/bash
# Round-4 pass AH: top launch lab, 16 waves (-DGS_TOP_E8=2: fourteen DMA waves,
# E on waves 0-7) against 8 (default) and 4 waves; then the top bitwise tests.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04ah
mkdir -p "$OUT"; cd "$ROOT"
for i in 1 2; do
  for V in base e8 e16; do
    echo "== $V tids round $i" >> "$OUT/top_lab_ab.txt"
    timeout -k 10 60 tools/bin/top_lab_$V tids >> "$OUT/top_lab_ab.txt" 2>&1 || exit $?
  done
done
grep -E "==|per launch|hash|stage" "$OUT/top_lab_ab.txt"
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_model.py \
    -k "top_launch or self_rows or deferred" > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"

#!/bin/bash
# Device sampler aux stream on/off, alternating, back-to-back batch time.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/ab_ds_aux
mkdir -p "$OUT"; cd "$ROOT"
for R in 1 2 3; do
  for V in 1 0; do
    timeout -k 10 200 env GS_DS_AUX=$V python -u tools/lab/ds_time.py > "$OUT/aux${V}_$R.log" 2>&1 || exit $?
    echo "aux=$V r$R: $(grep back-to-back "$OUT/aux${V}_$R.log")"
  done
done

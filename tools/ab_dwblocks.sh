#!/bin/bash
# A/B of the dW1 slab count (GS_DW_BLOCKS: target workgroups of the dW launch), alternating.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/ab_dw
mkdir -p "$OUT"; cd "$ROOT"
for rep in 1 2; do
  for b in 512 256 384 1024; do
    GS_DW_BLOCKS=$b timeout -k 10 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline > "$OUT/b${b}_$rep.json" 2>/dev/null || exit $?
    echo "blocks $b rep $rep: $(grep -o '"value": [0-9.]*' "$OUT/b${b}_$rep.json" | head -1)"
  done
done

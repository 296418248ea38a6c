#!/bin/bash
# Round-5 pass AH: forward lab, register-staged against LDS-DMA staged tiles
# (same binary: bitwise check of the second against the first).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd "$ROOT"
mkdir -p gpurun_out/r05ah
for i in G G4 G5; do
  echo "== fwd_lab_$i"; timeout -k 10 120 tools/bin/fwd_lab_$i 2>&1 | tee -a gpurun_out/r05ah/fwd_lab_G.txt || exit 1
done

#!/bin/bash
# Round-5 pass V: the dW lab with the odd-tail loop; slab heights 288 (the
# library's 16 slabs), 144 (32 slabs: two workgroups per CU), 320, 224; chunk 32.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd "$ROOT"
mkdir -p gpurun_out/r05v
for a in "4378" "4378 144" "4378 320" "4378 224" "4378 176"; do
  echo "== dw_lab $a"; timeout -k 10 120 tools/bin/dw_lab $a 2>&1 | tee -a gpurun_out/r05v/dw_lab.txt || exit 1
done
for v in dw_lab_c32 dw_lab_NO_STASH dw_lab_MFMA_ONLY; do
  echo "== $v"; timeout -k 10 120 tools/bin/$v 2>&1 | tee gpurun_out/r05v/$v.txt || exit 1
done

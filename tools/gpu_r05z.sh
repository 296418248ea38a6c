#!/bin/bash
# Round-5 pass Z: forward and dW labs, pipelined loops with and without a
# scheduling fence at the step boundaries (global-space lab stamps).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd "$ROOT"
mkdir -p gpurun_out/r05z
for v in fwd_lab fwd_lab_F fwd_lab_NO_MFMA dw_lab dw_lab_F; do
  echo "== $v"; timeout -k 10 120 tools/bin/$v 2>&1 | tee gpurun_out/r05z/$v.txt || exit 1
done

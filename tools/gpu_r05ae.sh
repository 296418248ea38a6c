#!/bin/bash
# Round-5 pass AE: wave priority (s_setprio 1) around the MFMA segments of the
# forward K loop and the dW row loop, lab A/B.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd "$ROOT"
mkdir -p gpurun_out/r05ae
for i in 1 2; do for v in fwd_lab fwd_lab_P dw_lab dw_lab_P; do
  echo "== $v"; timeout -k 10 120 tools/bin/$v 2>&1 | grep -v "fixed\|flushed" | tee -a gpurun_out/r05ae/$v.txt || exit 1
done; done

#!/bin/bash
# Round-5 pass AB: the forward lab, W in LDS (library) vs W in registers
# (linear_fwd_wreg_kernel), with and without step-boundary scheduling fences.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd "$ROOT"
mkdir -p gpurun_out/r05ab
for v in fwd_lab fwd_lab_W fwd_lab_WF; do
  echo "== $v"; timeout -k 10 120 tools/bin/$v 2>&1 | tee gpurun_out/r05ab/$v.txt || exit 1
done

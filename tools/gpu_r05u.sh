#!/bin/bash
# Round-5 pass U: dW lab ablations (no barrier / no operand reads / no stash),
# then the GPU model + kernel tests on the pipelined dW body.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd "$ROOT"
mkdir -p gpurun_out/r05u
for v in dw_lab dw_lab_NO_BARRIER dw_lab_NO_READ dw_lab_NO_STASH; do
  echo "== $v"; timeout -k 10 120 tools/bin/$v 2>&1 | tee gpurun_out/r05u/$v.txt || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05u/quick.log 2>&1; rc=$?
tail -3 gpurun_out/r05u/quick.log; exit $rc

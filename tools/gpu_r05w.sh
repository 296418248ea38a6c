#!/bin/bash
# Round-5 pass W: dW lab with LDS-only exchange barriers; hot-load ablation.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd "$ROOT"
mkdir -p gpurun_out/r05w
for v in dw_lab dw_lab_HOT; do
  echo "== $v"; timeout -k 10 120 tools/bin/$v 2>&1 | tee gpurun_out/r05w/$v.txt || exit 1
done

#!/bin/bash
# Round-5 pass AF: forward lab, the K loop without its loads and stash (MFMAs,
# LDS operand reads and barriers only) against the default.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd "$ROOT"
mkdir -p gpurun_out/r05af
for v in fwd_lab fwd_lab_NS; do
  echo "== $v"; timeout -k 10 120 tools/bin/$v 2>&1 | grep -v "fixed\|flushed" | tee -a gpurun_out/r05af/$v.txt || exit 1
done

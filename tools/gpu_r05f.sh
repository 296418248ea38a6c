#!/bin/bash
# Round-5 pass F: GPU suite on the dense-X2 + backward-records build, the top
# lab, then three alternating bench rounds: main, the committed 34c2812 build
# (c34), and main with forward prefetch depth 3 / 4 (fa3, fa4).
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r05f
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1; rc=$?
tail -5 "$OUT/gpu_tests.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 tools/bin/top_lab tids > "$OUT/top_lab.txt" 2>&1; rc=$?
tail -12 "$OUT/top_lab.txt"; [ $rc -ne 0 ] && exit $rc
P=graphsage-pytorch_amd
ROUNDS=3 timeout -k 10 1000 bash tools/ab_multi.sh $P/libgraphsage_amd.so $P/libgraphsage_amd_c34.so $P/libgraphsage_amd_fa3.so $P/libgraphsage_amd_fa4.so > "$OUT/ab.txt" 2>&1; rc=$?
cat "$OUT/ab.txt"; exit $rc

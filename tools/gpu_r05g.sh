#!/bin/bash
# Round-5 pass G: GPU suite on the forward with the branch-free prefetch ring
# (+ dense X2 + backward records), then a rocprof A/B against the committed
# 34c2812 build (c34) and the ring 3 / 4 chunks deep (fa3, fa4), two rounds.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd "$ROOT"
mkdir -p gpurun_out/r05g
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05g/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r05g/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
P=graphsage-pytorch_amd
OUT=gpurun_out/r05g ROUNDS=2 timeout -k 10 1000 bash tools/ab_prof.sh $P/libgraphsage_amd.so $P/libgraphsage_amd_c34.so $P/libgraphsage_amd_fa3.so $P/libgraphsage_amd_fa4.so

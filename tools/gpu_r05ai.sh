#!/bin/bash
# Round-5 pass: lookahead gather deferred behind the layer-1 forward.
# GPU suite, then rocprof A/B against the previous build, then plain bench A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05ai
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r05ai/gpu_tests.log 2>&1 && tail -2 gpurun_out/r05ai/gpu_tests.log &&
OUT=gpurun_out/r05ai/ab ROUNDS=2 bash tools/ab_prof.sh graphsage-pytorch_amd/libgraphsage_amd.so \
    graphsage-pytorch_amd/libgraphsage_amd_prev.so && tail -12 gpurun_out/r05ai/ab/runs.txt

#!/bin/bash
# Round-5 pass: the fused layer-1 dW + slab sum. Its bitwise test first, then
# the GPU suite, then rocprof A/B against the separate launches (prev.so =
# fused_dw1 off by default) and the plain bench A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ao
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -k fused_dw1 -x -v --timeout 120 --timeout-method thread > $O/fused_test.log 2>&1; rc=$?
tail -8 $O/fused_test.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 && tail -1 $O/gpu_tests.log &&
OUT=$O/ab ROUNDS=2 bash tools/ab_prof.sh graphsage-pytorch_amd/libgraphsage_amd.so graphsage-pytorch_amd/libgraphsage_amd_prev.so > $O/ab_summary.txt && grep median $O/ab_summary.txt &&
bash tools/ab_so.sh > $O/ab_so.txt 2>&1 && cat $O/ab_so.txt

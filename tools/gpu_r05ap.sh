#!/bin/bash
# Round-5 pass: fused dW1 with system-scope hand-off counters: its bitwise
# test, the full-size oracle test, then rocprof A/B and plain bench A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUTD:-r05ap}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_fullsize.py -k "fused_dw1 or runner_vs_oracle" -x -q --timeout 120 --timeout-method thread > $O/fused_test.log 2>&1; rc=$?
tail -3 $O/fused_test.log
[ $rc -eq 0 ] || exit 1
OUT=$O/ab ROUNDS=2 bash tools/ab_prof.sh graphsage-pytorch_amd/libgraphsage_amd.so graphsage-pytorch_amd/libgraphsage_amd_prev.so > $O/ab_summary.txt && grep median $O/ab_summary.txt &&
bash tools/ab_so.sh > $O/ab_so.txt 2>&1 && cat $O/ab_so.txt

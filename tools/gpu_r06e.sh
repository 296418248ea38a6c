#!/bin/bash
# r06 pass e: top lab v8 vs v10 (dIn on 8 waves, 8-byte W2 reads + ABID dZ); parity tests on v10; default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/r06e
mkdir -p $O
for v in v8 v10 v8 v10; do
  timeout -k 10 120 tools/bin/top_lab_$v tids > $O/top_lab_$v.txt 2>&1; echo "lab $v rc=$?"; grep "v2 top kernel\|v2:" $O/top_lab_$v.txt | tail -2; grep -A10 "stamped launch 2" $O/top_lab_$v.txt
done
TESTS="tests/test_gpu_model.py tests/test_gpu_dp.py tests/test_gpu_fullsize.py::test_fullsize_timed_step_fp32_max_vs_oracle tests/test_gpu_fullsize.py::test_fullsize_timed_step_embeddings_and_grads_vs_oracle tests/test_gpu_fullsize.py::test_fullsize_timed_step_bf16_max_vs_oracle" \
  BENCH=default TAG=r06e bash tools/gpu_pass.sh

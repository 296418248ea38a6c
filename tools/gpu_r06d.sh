#!/bin/bash
# r06 pass d: forward lab with / without K-chunk rotation; top lab v7 / v8 / v9; the top / step parity tests on the new kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/r06d
mkdir -p $O
for b in fwd_lab fwd_lab_rot fwd_lab fwd_lab_rot; do
  timeout -k 10 120 tools/bin/$b > $O/$b.txt 2>&1; echo "$b rc=$?"; grep "per launch\|stamps" $O/$b.txt | head -6
done
for v in v7 v8 v9 v8 v9; do
  timeout -k 10 120 tools/bin/top_lab_$v tids > $O/top_lab_$v.txt 2>&1; echo "lab $v rc=$?"; grep "v2 top kernel\|v2:" $O/top_lab_$v.txt | tail -2; grep -A10 "stamped launch 2" $O/top_lab_$v.txt
done
timeout -k 10 120 tools/bin/top_lab_v9 > $O/top_lab_v9_ptr.txt 2>&1; echo "lab v9 (ptr lists) rc=$?"; grep "v2 top kernel\|v2:" $O/top_lab_v9_ptr.txt | tail -2
TESTS="tests/test_gpu_model.py tests/test_gpu_dp.py tests/test_gpu_fullsize.py::test_fullsize_timed_step_fp32_max_vs_oracle tests/test_gpu_fullsize.py::test_fullsize_timed_step_embeddings_and_grads_vs_oracle tests/test_gpu_fullsize.py::test_fullsize_timed_step_bf16_max_vs_oracle" \
  TAG=r06d bash tools/gpu_pass.sh

#!/bin/bash
# r06 pass b: top lab probes (v4 = loss-head operands on the DMA waves; nos = v4 without slab stores),
# then the deferred W=2 and full-size timed-step tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}"
mkdir -p gpurun_out/r06b
for b in top_lab_v4 top_lab_v4_nos; do
  timeout -k 10 120 tools/bin/$b tids > gpurun_out/r06b/$b.txt 2>&1; echo "$b rc=$?"; grep "per launch\|err" gpurun_out/r06b/$b.txt | tail -3; grep -A12 "stamped launch 2" gpurun_out/r06b/$b.txt
done
TESTS="tests/test_gpu_dp.py tests/test_gpu_fullsize.py::test_fullsize_timed_step_fp32_max_vs_oracle tests/test_gpu_fullsize.py::test_fullsize_timed_step_embeddings_and_grads_vs_oracle" \
  TAG=r06b bash tools/gpu_pass.sh

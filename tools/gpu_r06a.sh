#!/bin/bash
# r06 first pass: the top lab probes, the new parity tests + top tests, the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}"
mkdir -p gpurun_out/r06a
for b in top_lab top_lab_nodma top_lab_v3; do
  timeout -k 10 120 tools/bin/$b tids > gpurun_out/r06a/$b.txt 2>&1; echo "$b rc=$?"; grep "per launch\|err" gpurun_out/r06a/$b.txt | head -4; grep -A12 "stamped launch 2" gpurun_out/r06a/$b.txt
done
TESTS="tests/test_gpu_dp.py tests/test_gpu_model.py -k top tests/test_gpu_fullsize.py::test_fullsize_timed_step_fp32_max_vs_oracle tests/test_gpu_fullsize.py::test_fullsize_timed_step_embeddings_and_grads_vs_oracle" \
  BENCH=default TAG=r06a bash tools/gpu_pass.sh

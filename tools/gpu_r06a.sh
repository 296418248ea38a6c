#!/bin/bash
# r06 first pass: the new parity tests, the top lab with fine stage stamps, the default bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}"
mkdir -p gpurun_out/r06a
timeout -k 10 120 tools/bin/top_lab tids > gpurun_out/r06a/top_lab.txt 2>&1; echo "top_lab rc=$?"; cat gpurun_out/r06a/top_lab.txt | tail -40
TESTS="tests/test_gpu_dp.py tests/test_gpu_fullsize.py::test_fullsize_timed_step_fp32_max_vs_oracle tests/test_gpu_fullsize.py::test_fullsize_timed_step_embeddings_and_grads_vs_oracle" \
  BENCH=default TAG=r06a bash tools/gpu_pass.sh

#!/bin/bash
# Round-5 pass X: the pipelined dW body in the library: quick tests, site 2 / 4
# stamps, rocprof A/B against the previous commit's build.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd "$ROOT"
mkdir -p gpurun_out/r05x
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05x/quick.log 2>&1; rc=$?
tail -3 gpurun_out/r05x/quick.log; [ $rc -ne 0 ] && exit $rc
for s in 2 4; do
  timeout -k 10 300 python -u tools/lab/site_stamps.py $s 40 > gpurun_out/r05x/stamps_$s.txt 2>&1; rc=$?
  tail -12 gpurun_out/r05x/stamps_$s.txt; [ $rc -ne 0 ] && exit $rc
done
OUT=gpurun_out/r05x/ab ROUNDS=2 timeout -k 10 1500 bash tools/ab_prof.sh graphsage-pytorch_amd/libgraphsage_amd.so graphsage-pytorch_amd/libgraphsage_amd_prev.so || exit 1

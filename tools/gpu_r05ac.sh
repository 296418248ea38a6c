#!/bin/bash
# Round-5 pass AC: the layer-2 slab sum on split blocks: the GPU suite,
# site 2 / 4 stamps, rocprof A/B against the previous commit's build.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd "$ROOT"
mkdir -p gpurun_out/r05ac
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ac/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r05ac/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
for s in 4; do
  timeout -k 10 300 python -u tools/lab/site_stamps.py $s 40 > gpurun_out/r05ac/stamps_$s.txt 2>&1; rc=$?
  tail -12 gpurun_out/r05ac/stamps_$s.txt; [ $rc -ne 0 ] && exit $rc
done
OUT=gpurun_out/r05ac/ab ROUNDS=2 timeout -k 10 1500 bash tools/ab_prof.sh graphsage-pytorch_amd/libgraphsage_amd.so graphsage-pytorch_amd/libgraphsage_amd_prev.so || exit 1
timeout -k 10 300 python -u tools/lab/pubmed_phases.py pubmed 7 > gpurun_out/r05ac/pubmed_phases.txt 2>&1; rc=$?
tail -3 gpurun_out/r05ac/pubmed_phases.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --config pubmed --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/r05ac/bench_pubmed.log 2>&1; rc=$?
tail -1 gpurun_out/r05ac/bench_pubmed.log | cut -c1-400; exit $rc

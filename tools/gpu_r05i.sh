#!/bin/bash
# Round-5 pass I: GPU suite with the balanced forward row split, then
# alternating bench runs (workgroup stamp statistics) and a rocprof A/B
# against the previous commit's build (prev).
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd "$ROOT"
mkdir -p gpurun_out/r05i
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05i/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r05i/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
P=graphsage-pytorch_amd
cp $P/libgraphsage_amd.so /tmp/lib_main.so
for i in 1 2; do
  for so in /tmp/lib_main.so $P/libgraphsage_amd_prev.so; do
    cp $so $P/libgraphsage_amd.so
    timeout -k 10 300 python bench.py --steps 300 --warmup 10 --sustain 300 --no-cpu-baseline --ref-stream-steps 0 > gpurun_out/r05i/bench.log 2>&1 || { cp /tmp/lib_main.so $P/libgraphsage_amd.so; exit 1; }
    python3 -c "import json,sys;d=json.loads([x for x in open('gpurun_out/r05i/bench.log').read().splitlines() if x.startswith('{')][-1]);print(sys.argv[1], d['ms_per_step'], d['sustained']['ms_per_step']);[print('  ', k, v['avg_launch_us'], v.get('workgroup_us')) for k,v in d['roofline_kernels'].items()]" $(basename $so)
  done
done
cp /tmp/lib_main.so $P/libgraphsage_amd.so
OUT=gpurun_out/r05i ROUNDS=2 timeout -k 10 1000 bash tools/ab_prof.sh $P/libgraphsage_amd.so $P/libgraphsage_amd_prev.so

#!/bin/bash
# Round-5 pass H: the per-workgroup stamp statistics (test + one bench line).
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd "$ROOT"
mkdir -p gpurun_out/r05h
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -k "kernel_timer" -x -q --timeout 120 --timeout-method thread > gpurun_out/r05h/test.log 2>&1; rc=$?
tail -3 gpurun_out/r05h/test.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 300 --warmup 10 --sustain 300 --no-cpu-baseline --ref-stream-steps 0 > gpurun_out/r05h/bench$i.log 2>&1 || exit 1
python3 -c "import json;d=json.loads([x for x in open('gpurun_out/r05h/bench$i.log').read().splitlines() if x.startswith('{')][-1]);print(d['ms_per_step'], d['sustained']['ms_per_step']);[print(k, v['avg_launch_us'], v.get('workgroup_us')) for k,v in d['roofline_kernels'].items()]"
done

#!/bin/bash
# A/B: fence-free timer + runner events (default) against system-fenced ones.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/ab_fence
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_dp.py tests/test_gpu_fullsize.py -q -k "runner or dp or bucket or held" \
    -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for mode in nofence fence; do
    if [ $mode = fence ]; then export GS_TIMER_SYSFENCE=1 GS_RUNNER_SYSFENCE=1; else unset GS_TIMER_SYSFENCE GS_RUNNER_SYSFENCE; fi
    timeout -k 10 200 python bench.py --steps ${STEPS:-300} --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > "$OUT/b_${mode}_$i.log" 2>&1 || exit $?
    python3 -c "
import json,sys; d=json.loads(open('$OUT/b_${mode}_$i.log').read().strip().splitlines()[-1]); r=d['roofline_kernels']
print('$mode', d['value'], d['ms_per_step'], 'sus', (d.get('sustained') or {}).get('value'), {k:v['avg_launch_us'] for k,v in r.items()}, d['roofline']['kernel'][:40])"
  done
done

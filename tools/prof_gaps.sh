#!/bin/bash
# rocprofv3 kernel traces of the bench under two runtime modes (A/B of event fences), for step-gap analysis.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/gaps
mkdir -p "$OUT"
cd "$ROOT"
for mode in ${MODES:-nofence fence}; do
  if [ $mode = fence ]; then export GS_TIMER_SYSFENCE=1 GS_RUNNER_SYSFENCE=1; else unset GS_TIMER_SYSFENCE GS_RUNNER_SYSFENCE; fi
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/$mode" -o run --output-format csv -- \
      python3 bench.py --steps 100 --warmup 5 --sustain 100 --no-cpu-baseline ${BENCH_ARGS} > "$OUT/$mode.log" 2>&1 || exit $?
  tail -1 "$OUT/$mode.log" | cut -c1-200
done

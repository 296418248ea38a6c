#!/bin/bash
# Sampler stream / helper-thread layouts on the bench workload (20-step cold
# start and 300 steps), one box session.  LAYOUTS: "S:H S:H ..." (streams,
# helpers per stream).  Stops at the first failing run.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/${TAG:-ab_sampler}
mkdir -p "$OUT"
cd "$ROOT"
for lay in ${LAYOUTS:-12:0 6:1 4:2 1:0 1:3}; do
  S=${lay%%:*}; HH=${lay##*:}
  for steps in ${STEPS:-20 300}; do
    timeout -k 10 240 python bench.py --steps $steps --warmup 5 --no-cpu-baseline --sustain 0 \
        --sampler-streams $S --sampler-helpers $HH ${BENCH_ARGS} > "$OUT/s${S}_h${HH}_k$steps.log" 2>&1 || exit $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], sys.argv[4], d['value'], d['ms_per_step'], d['config']['host_ms_per_step']['sampler'])" "$OUT/s${S}_h${HH}_k$steps.log" $S $HH $steps
  done
done

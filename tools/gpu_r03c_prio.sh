#!/bin/bash
# Device sampler stream priority A/B (high = default, GS_DS_PRIO=0 normal),
# S = 1 and S = 4, alternating.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r03c_prio
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    tests/test_gpu_fullsize.py tests/test_gpu_model.py -k "device" > "$OUT/tests.log" 2>&1
rc=$?; tail -2 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
for S in 1 4; do
  for R in 1 2; do
    for V in "" "GS_DS_PRIO=0"; do
      N=s${S}_${V:-hi}_$R
      timeout -k 10 300 env $V python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --sampler device --sampler-streams $S > "$OUT/$N.json" 2> "$OUT/$N.err" || exit $?
      echo "$N: $(grep -o '"value": [0-9.]*' "$OUT/$N.json" | head -1)"
    done
  done
done

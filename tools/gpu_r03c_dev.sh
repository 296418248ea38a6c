#!/bin/bash
# Device-runner depth A/B: the device-sampler tests, then the S = 1 device line
# with two runs queued per stream (default) and one (GS_DS_DEPTH=1), and the
# S = 4 line with and without the aux stream.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r03c_dev
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
    tests/test_gpu_dsampler.py tests/test_gpu_fullsize.py tests/test_gpu_model.py -k "dsampler or device or aux" > "$OUT/tests.log" 2>&1
rc=$?; tail -2 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
for R in 1 2; do
  for V in "" "GS_DS_DEPTH=1"; do
    timeout -k 10 300 env $V python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --sampler device --sampler-streams 1 > "$OUT/s1_${V:-d2}_$R.json" 2> "$OUT/s1_${V:-d2}_$R.err" || exit $?
    echo "S=1 ${V:-depth2} r$R: $(grep -o '"value": [0-9.]*' "$OUT/s1_${V:-d2}_$R.json" | head -1)"
  done
done
for V in "" "GS_DS_AUX=0"; do
  timeout -k 10 300 env $V python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --sampler device --sampler-streams 4 > "$OUT/s4_${V:-aux}.json" 2> "$OUT/s4_${V:-aux}.err" || exit $?
  echo "S=4 ${V:-aux}: $(grep -o '"value": [0-9.]*' "$OUT/s4_${V:-aux}.json" | head -1)"
done

#!/bin/bash
# Round-3 GPU pass A: the new parity tests (rmat16m full size, empty device
# balls), the touched paths, then the driver's bench command twice and a
# 300-step line with the sustained window's new fields.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r03a
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 400 --timeout-method thread \
    tests/test_gpu_unsup_ball.py tests/test_gpu_dp.py tests/test_gpu_fullsize16m.py -s > "$OUT/tests.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
run() {  # name, args
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err"
  local rc=$?; echo "bench $name rc=$rc"; tail -c 300 "$OUT/bench_$name.json"; echo; return $rc
}
run d1 --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
run d2 --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
run s300 --gpus 1 --steps 300 --warmup 5 --no-cpu-baseline || exit $?
run s300_h0 --gpus 1 --steps 300 --warmup 5 --no-cpu-baseline --sampler-helpers 0 || exit $?

#!/bin/bash
# Device-sampler training path: parity tests, then bench lines (device S=1,
# S=2, and the host S=1 reference-sequence mode for comparison).
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/${TAG:-r03b}
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    tests/test_gpu_dsampler.py tests/test_gpu_fullsize.py -k "device or replays" > "$OUT/tests.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
run() {  # name, args
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err"
  local rc=$?; echo "bench $name rc=$rc"; python3 -c "
import json,sys; d=json.loads(open('$OUT/bench_$name.json').read().strip().splitlines()[-1]); c=d['config']
print(d['value'], d['ms_per_step'], 'sus', (d.get('sustained') or {}).get('value'), c['sampler'])" ; return $rc
}
run dev_s1 --gpus 1 --steps 100 --warmup 5 --no-cpu-baseline --sampler device --sustain 100 || exit $?
run dev_s2 --gpus 1 --steps 100 --warmup 5 --no-cpu-baseline --sampler device --sampler-streams 2 --sustain 100 || exit $?
run host_s1 --gpus 1 --steps 100 --warmup 5 --no-cpu-baseline --sampler-streams 1 --sampler-helpers 7 --sustain 100 || exit $?

#!/bin/bash
# Round-3 final check of the committed build: the -m gpu suite, smoke(), the
# device-sampler lines (S = 1 / 4) and the device sampler's kernel stats.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r03c_final
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -2 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
echo smoke ok
for S in 1 4; do
  timeout -k 10 300 python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --sampler device --sampler-streams $S > "$OUT/bench_rmat2m_device_s$S.json" 2> "$OUT/bench_rmat2m_device_s$S.err" || exit $?
  echo "device S=$S: $(grep -o '"value": [0-9.]*' "$OUT/bench_rmat2m_device_s$S.json" | head -1)"
done
TAG=r03c_final/ds bash tools/gpu_ds.sh > "$OUT/ds.log" 2>&1 || exit $?
grep -E "latency|back-to-back" "$OUT/ds.log"

#!/bin/bash
# Round-4 first pass: the -m gpu suite on the bounded-loop build (plus the
# new full-size parity tests), smoke(), the driver's default bench command.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04a
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
echo smoke ok
timeout -k 10 400 python3 bench.py > "$OUT/bench_rmat2m_steps20.json" 2> "$OUT/bench_rmat2m_steps20.err" || exit $?
echo "default: $(grep -o '"value": [0-9.]*' "$OUT/bench_rmat2m_steps20.json" | head -1)"

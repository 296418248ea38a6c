#!/bin/bash
# Round-3 re-entry check: the -m gpu suite and the driver's default bench
# command on the restored tree.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r03re
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --no-cpu-baseline > "$OUT/bench_rmat2m_steps20.json" 2> "$OUT/bench_rmat2m_steps20.err" || exit $?
grep -o '"value": [0-9.]*' "$OUT/bench_rmat2m_steps20.json" | head -1

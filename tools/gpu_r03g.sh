#!/bin/bash
# Headline bench: default line, a 300-step line, and its rocprof kernel stats.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/${TAG:-r03g}
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 400 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || exit $?
tail -c 300 "$OUT/bench_default.json"; echo
timeout -k 10 400 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --sustain 300 > "$OUT/bench_300.json" 2> "$OUT/bench_300.err" || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --steps 300 --warmup 5 --no-cpu-baseline --sustain 300 > "$OUT/prof.log" 2>&1 || exit $?

#!/bin/bash
# Round-5 pass A: baseline of the round-4 build on this round's box: the
# default bench line and rocprofv3 kernel stats of the 300-step fp32 bench.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r05a
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || exit $?
tail -c 600 "$OUT/bench_default.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_rmat2m" -o run --output-format csv -- python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --ref-stream-steps 0 > "$OUT/prof_rmat2m.log" 2>&1 || exit $?
cp "$OUT/prof_rmat2m/run_kernel_stats.csv" "$OUT/kernel_stats_rmat2m_steps300.csv" || exit 1
rm -rf "$OUT/prof_rmat2m"
head -20 "$OUT/kernel_stats_rmat2m_steps300.csv" | cut -c1-200

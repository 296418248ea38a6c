#!/bin/bash
# Round-3 pass A: the whole -m gpu suite, smoke(), the headline's rocprofv3
# kernel stats (copied into profiles/ first, so the bench lines that follow
# cite them), the driver's default command and a 300-step line.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r03final
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
echo smoke ok
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_rmat2m" -o run --output-format csv -- python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline > "$OUT/prof_rmat2m.log" 2>&1 || exit $?
cp "$OUT/prof_rmat2m/run_kernel_stats.csv" profiles/r03_kernel_stats_rmat2m_steps300.csv || exit 1
timeout -k 10 400 python3 bench.py > "$OUT/bench_rmat2m_steps20.json" 2> "$OUT/bench_rmat2m_steps20.err" || exit $?
tail -c 400 "$OUT/bench_rmat2m_steps20.json"; echo
timeout -k 10 400 python3 bench.py --steps 300 --warmup 5 --sustain 300 > "$OUT/bench_rmat2m_steps300.json" 2> "$OUT/bench_rmat2m_steps300.err" || exit $?
grep -o '"value": [0-9.]*' "$OUT/bench_rmat2m_steps300.json" | head -1

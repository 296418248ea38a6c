#!/bin/bash
# Round-3 second measurement pass, part A: the -m gpu suite, smoke(), the
# headline's rocprofv3 kernel stats (into profiles/ first, so the bench lines
# cite them), the driver's default command, a 300-step line, bf16 MAX.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r03b
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -2 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
echo smoke ok
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_rmat2m" -o run --output-format csv -- python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline > "$OUT/prof_rmat2m.log" 2>&1 || exit $?
cp "$OUT/prof_rmat2m/run_kernel_stats.csv" profiles/r03b_kernel_stats_rmat2m_steps300.csv || exit 1
timeout -k 10 400 python3 bench.py > "$OUT/bench_rmat2m_steps20.json" 2> "$OUT/bench_rmat2m_steps20.err" || exit $?
echo "default: $(grep -o '"value": [0-9.]*' "$OUT/bench_rmat2m_steps20.json" | head -1)"
timeout -k 10 400 python3 bench.py --steps 300 --warmup 5 --sustain 300 > "$OUT/bench_rmat2m_steps300.json" 2> "$OUT/bench_rmat2m_steps300.err" || exit $?
echo "300: $(grep -o '"value": [0-9.]*' "$OUT/bench_rmat2m_steps300.json" | head -1)"
C=rmat2m-max-bf16; N=rmat2m_max_bf16
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$N" -o run --output-format csv -- python3 bench.py --config $C --steps 300 --warmup 5 --no-cpu-baseline > "$OUT/prof_$N.log" 2>&1 || exit $?
cp "$OUT/prof_$N/run_kernel_stats.csv" "profiles/r03b_kernel_stats_${N}_steps300.csv" || exit 1
timeout -k 10 500 python3 bench.py --config $C --steps 300 --warmup 5 --sustain 300 > "$OUT/bench_${N}_steps300.json" 2> "$OUT/bench_${N}_steps300.err" || exit $?
echo "$C: $(grep -o '"value": [0-9.]*' "$OUT/bench_${N}_steps300.json" | head -1)"

#!/bin/bash
# Round-3 third measurement pass, part A (current build: 48-row layer-1
# forward tiles, device sampler aux stream): the -m gpu suite, smoke(), the
# headline's rocprofv3 kernel stats and PMC HBM traffic (into profiles/ first,
# so the bench lines cite them), the driver's default command, 300 steps.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r03c
mkdir -p "$OUT/pmc"; cd "$ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$OUT/gpu_tests.log" 2>&1
rc=$?; tail -2 "$OUT/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
cp "$OUT/gpu_tests.log" profiles/r03c_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
echo smoke ok
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_rmat2m" -o run --output-format csv -- python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline > "$OUT/prof_rmat2m.log" 2>&1 || exit $?
cp "$OUT/prof_rmat2m/run_kernel_stats.csv" profiles/r03c_kernel_stats_rmat2m_steps300.csv || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $C -d "$OUT/pmc/$C" -o run --output-format csv -- \
      python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --sustain 0 > "$OUT/pmc/bench_$C.log" 2>&1 || exit $?
done
python3 tools/pmc_summary.py "$OUT/pmc" rmat2m > "$OUT/pmc_traffic_rmat2m.json" || exit $?
cp "$OUT/pmc_traffic_rmat2m.json" profiles/r03c_pmc_traffic_rmat2m.json
echo pmc ok
timeout -k 10 400 python3 bench.py > "$OUT/bench_rmat2m_steps20.json" 2> "$OUT/bench_rmat2m_steps20.err" || exit $?
echo "default: $(grep -o '"value": [0-9.]*' "$OUT/bench_rmat2m_steps20.json" | head -1)"
timeout -k 10 400 python3 bench.py --steps 300 --warmup 5 --sustain 300 > "$OUT/bench_rmat2m_steps300.json" 2> "$OUT/bench_rmat2m_steps300.err" || exit $?
echo "300: $(grep -o '"value": [0-9.]*' "$OUT/bench_rmat2m_steps300.json" | head -1)"

#!/bin/bash
# Round-3 third measurement pass, part B: bf16 MAX (rocprof + line), the
# sampler lines (device S = 1 / 4, host S = 1 with helpers), the device
# sampler's kernel stats, Pubmed.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r03c
mkdir -p "$OUT"; cd "$ROOT"
C=rmat2m-max-bf16; N=rmat2m_max_bf16
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$N" -o run --output-format csv -- python3 bench.py --config $C --steps 300 --warmup 5 --no-cpu-baseline > "$OUT/prof_$N.log" 2>&1 || exit $?
cp "$OUT/prof_$N/run_kernel_stats.csv" "profiles/r03c_kernel_stats_${N}_steps300.csv" || exit 1
timeout -k 10 500 python3 bench.py --config $C --steps 300 --warmup 5 --sustain 300 > "$OUT/bench_${N}_steps300.json" 2> "$OUT/bench_${N}_steps300.err" || exit $?
echo "$C: $(grep -o '"value": [0-9.]*' "$OUT/bench_${N}_steps300.json" | head -1)"
timeout -k 10 400 python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --sampler device --sampler-streams 1 > "$OUT/bench_rmat2m_device_s1.json" 2> "$OUT/bench_rmat2m_device_s1.err" || exit $?
echo "device S=1: $(grep -o '"value": [0-9.]*' "$OUT/bench_rmat2m_device_s1.json" | head -1)"
timeout -k 10 400 python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --sampler device --sampler-streams 4 > "$OUT/bench_rmat2m_device_s4.json" 2> "$OUT/bench_rmat2m_device_s4.err" || exit $?
echo "device S=4: $(grep -o '"value": [0-9.]*' "$OUT/bench_rmat2m_device_s4.json" | head -1)"
timeout -k 10 400 python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --sampler-streams 1 --sampler-helpers 7 > "$OUT/bench_rmat2m_s1_h7.json" 2> "$OUT/bench_rmat2m_s1_h7.err" || exit $?
echo "host S=1 h7: $(grep -o '"value": [0-9.]*' "$OUT/bench_rmat2m_s1_h7.json" | head -1)"
timeout -k 10 400 python3 bench.py --config pubmed --steps 40 --warmup 3 > "$OUT/bench_pubmed_apply_model.json" 2> "$OUT/bench_pubmed.err" || exit $?
echo "pubmed: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_pubmed_apply_model.json" | head -1)"
TAG=r03c/ds bash tools/gpu_ds.sh > "$OUT/ds.log" 2>&1 || exit $?
grep -E "latency|back-to-back" "$OUT/ds.log"

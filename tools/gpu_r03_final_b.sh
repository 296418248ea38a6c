#!/bin/bash
# Round-3 pass B: configs[3] (bf16 MAX) and configs[4] (rmat16m) — rocprofv3
# stats first (into profiles/), then their 300-step lines — and the sampler
# lines (device sampler S=4 / S=1, host S=1 with helpers).
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r03final
mkdir -p "$OUT"; cd "$ROOT"
for C in rmat2m-max-bf16 rmat16m; do
  N=$(echo $C | tr '-' '_')
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$N" -o run --output-format csv -- python3 bench.py --config $C --steps 300 --warmup 5 --no-cpu-baseline > "$OUT/prof_$N.log" 2>&1 || exit $?
  cp "$OUT/prof_$N/run_kernel_stats.csv" "profiles/r03_kernel_stats_${N}_steps300.csv" || exit 1
  timeout -k 10 500 python3 bench.py --config $C --steps 300 --warmup 5 --sustain 300 > "$OUT/bench_${N}_steps300.json" 2> "$OUT/bench_${N}_steps300.err" || exit $?
  echo "$C: $(grep -o '"value": [0-9.]*' "$OUT/bench_${N}_steps300.json" | head -1)"
done
timeout -k 10 400 python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --sampler device --sampler-streams 4 > "$OUT/bench_rmat2m_device_s4.json" 2> "$OUT/bench_rmat2m_device_s4.err" || exit $?
echo "device S=4: $(grep -o '"value": [0-9.]*' "$OUT/bench_rmat2m_device_s4.json" | head -1)"
timeout -k 10 400 python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --sampler device --sampler-streams 1 > "$OUT/bench_rmat2m_device_s1.json" 2> "$OUT/bench_rmat2m_device_s1.err" || exit $?
echo "device S=1: $(grep -o '"value": [0-9.]*' "$OUT/bench_rmat2m_device_s1.json" | head -1)"
timeout -k 10 400 python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --sampler-streams 1 --sampler-helpers 7 > "$OUT/bench_rmat2m_s1_h7.json" 2> "$OUT/bench_rmat2m_s1_h7.err" || exit $?
echo "host S=1 h7: $(grep -o '"value": [0-9.]*' "$OUT/bench_rmat2m_s1_h7.json" | head -1)"

#!/bin/bash
# Round-3 second measurement pass, part B: sampler lines (device S = 1 / 4,
# host S = 1 with helpers), the device sampler's kernel stats, Pubmed, and the
# headline's PMC HBM traffic.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r03b
mkdir -p "$OUT/pmc"; cd "$ROOT"
timeout -k 10 500 python3 bench.py --config rmat2m-max-bf16 --steps 300 --warmup 5 --sustain 300 > "$OUT/bench_rmat2m_max_bf16_steps300_b.json" 2> "$OUT/bench_rmat2m_max_bf16_steps300_b.err" || exit $?
echo "bf16 again: $(grep -o '"value": [0-9.]*' "$OUT/bench_rmat2m_max_bf16_steps300_b.json" | head -1)"
timeout -k 10 400 python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --sampler device --sampler-streams 1 > "$OUT/bench_rmat2m_device_s1.json" 2> "$OUT/bench_rmat2m_device_s1.err" || exit $?
echo "device S=1: $(grep -o '"value": [0-9.]*' "$OUT/bench_rmat2m_device_s1.json" | head -1)"
timeout -k 10 400 python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --sampler device --sampler-streams 4 > "$OUT/bench_rmat2m_device_s4.json" 2> "$OUT/bench_rmat2m_device_s4.err" || exit $?
echo "device S=4: $(grep -o '"value": [0-9.]*' "$OUT/bench_rmat2m_device_s4.json" | head -1)"
timeout -k 10 400 python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --sampler-streams 1 --sampler-helpers 7 > "$OUT/bench_rmat2m_s1_h7.json" 2> "$OUT/bench_rmat2m_s1_h7.err" || exit $?
echo "host S=1 h7: $(grep -o '"value": [0-9.]*' "$OUT/bench_rmat2m_s1_h7.json" | head -1)"
timeout -k 10 400 python3 bench.py --config pubmed --steps 40 --warmup 3 > "$OUT/bench_pubmed_apply_model.json" 2> "$OUT/bench_pubmed.err" || exit $?
echo "pubmed: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_pubmed_apply_model.json" | head -1)"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $C -d "$OUT/pmc/$C" -o run --output-format csv -- \
      python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --sustain 0 > "$OUT/pmc/bench_$C.log" 2>&1 || exit $?
done
python3 tools/pmc_summary.py "$OUT/pmc" rmat2m > "$OUT/pmc_traffic_rmat2m.json" || exit $?
echo pmc ok
TAG=r03b/ds bash tools/gpu_ds.sh > "$OUT/ds.log" 2>&1 || exit $?
grep -E "latency|back-to-back" "$OUT/ds.log"

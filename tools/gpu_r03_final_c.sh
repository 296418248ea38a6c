#!/bin/bash
# Round-3 pass C: the apply_model lines (pubmed with its CPU baseline, cora),
# full-graph inference, HBM traffic of the headline (separate --pmc passes)
# and the device sampler's kernel stats.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r03final
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 400 python3 bench.py --config pubmed --steps 40 --warmup 3 > "$OUT/bench_pubmed_apply_model.json" 2> "$OUT/bench_pubmed.err" || exit $?
echo "pubmed: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_pubmed_apply_model.json" | head -1)"
timeout -k 10 400 python3 bench.py --config cora --steps 40 --warmup 3 > "$OUT/bench_cora_apply_model.json" 2> "$OUT/bench_cora.err" || exit $?
echo "cora: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_cora_apply_model.json" | head -1)"
timeout -k 10 400 python3 bench.py --config rmat2m-embed --full-graph --no-cpu-baseline > "$OUT/bench_rmat2m_embed_full_graph.json" 2> "$OUT/bench_embed.err" || exit $?
echo "embed: $(grep -o '"value": [0-9.]*' "$OUT/bench_rmat2m_embed_full_graph.json" | head -1)"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $C -d "$OUT/pmc/$C" -o run --output-format csv -- \
      python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --sustain 0 > "$OUT/pmc/bench_$C.log" 2>&1 || exit $?
done
python3 tools/pmc_summary.py "$OUT/pmc" rmat2m > "$OUT/pmc_traffic_rmat2m.json" || exit $?
TAG=r03final/ds bash tools/gpu_ds.sh > "$OUT/ds.log" 2>&1 || exit $?
tail -30 "$OUT/ds.log" | grep -E "latency|back-to-back"

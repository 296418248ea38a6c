#!/bin/bash
# Host-side profile of the Pubmed apply_model loop (cProfile), host and device forward sampler.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/pubprof
mkdir -p "$OUT"; cd "$ROOT"
for s in host device; do
  timeout -k 10 300 python -m cProfile -o "$OUT/$s.prof" bench.py --config pubmed --steps 40 --warmup 3 --no-cpu-baseline --sampler $s > "$OUT/$s.json" 2> "$OUT/$s.err" || exit $?
  python -c "import pstats; p=pstats.Stats('$OUT/$s.prof'); p.sort_stats('cumulative').print_stats(45); p.sort_stats('tottime').print_stats(30)" > "$OUT/$s.txt" || exit $?
  tail -c 400 "$OUT/$s.json"; echo
done

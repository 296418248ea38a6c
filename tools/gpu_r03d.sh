#!/bin/bash
# Pubmed outliers: classifier slab sum (rows per block grown with B) and the
# pulled ball BFS; parity tests first, then the Pubmed bench and its profile.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/${TAG:-r03d}
mkdir -p "$OUT"
cd "$ROOT"
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_unsup_ball.py tests/test_gpu_pubmed.py > "$OUT/tests.log" 2>&1
rc=$?; [ -n "$SKIP_TESTS" ] || { tail -5 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc; }
timeout -k 10 300 python bench.py --config pubmed --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/bench_pub.json" 2> "$OUT/bench_pub.err" || exit $?
tail -c 800 "$OUT/bench_pub.json"; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_pub" -o run --output-format csv -- python bench.py --config pubmed --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/prof_pub.log" 2>&1 || exit $?
find "$OUT/prof_pub" -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} "$OUT/kernel_stats_pub.csv"
head -14 "$OUT/kernel_stats_pub.csv" | cut -c1-160

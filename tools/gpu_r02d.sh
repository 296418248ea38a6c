#!/bin/bash
# rocprofv3 kernel stats of the bf16 MAX and rmat16m 300-step bench commands,
# then their bench lines with those stats in place (bench.py prices the
# kernel with the largest rocprof average as the dominant one).
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r02d
mkdir -p "$OUT"
cd "$ROOT"
for pair in "rmat2m-max-bf16:rmat2m_max_bf16" "rmat16m:rmat16m"; do
  cfg=${pair%%:*}; tag=${pair##*:}
  mkdir -p "$OUT/prof_$tag"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$tag" -o run --output-format csv -- \
      python3 bench.py --config "$cfg" --steps 300 --warmup 5 --no-cpu-baseline > "$OUT/prof_$tag/bench.json" 2> "$OUT/prof_$tag/bench.err"
  rc=$?; echo "rocprof $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
  rm -f "$OUT/prof_$tag/run_kernel_trace.csv"
  cp "$OUT/prof_$tag/run_kernel_stats.csv" "profiles/r02_kernel_stats_${tag}_steps300.csv" || exit 1
  timeout -k 10 300 python bench.py --config "$cfg" --steps 300 --warmup 5 --no-cpu-baseline > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err"
  rc=$?; echo "bench $cfg rc=$rc"; tail -c 300 "$OUT/bench_$tag.json"; echo; [ $rc -eq 0 ] || exit $rc
done

#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench run (no PMC counters here).
set -o pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$PWD}/gpurun_out/prof_${TAG:-trace}
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-$PWD}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- \
    python3 bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > "$OUT/bench.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 "$OUT/bench.log"
find "$OUT" -name "*stats*.csv" | head
exit $rc

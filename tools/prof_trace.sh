#!/bin/bash
# rocprofv3 kernel + memory-copy trace of a short bench run (timeline analysis).
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/trace_${TAG:-x}
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT" -o run --output-format csv -- \
    python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > "$OUT/bench.log" 2>&1
rc=$?; tail -1 "$OUT/bench.log"; exit $rc

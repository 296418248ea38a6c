#!/bin/bash
# One rocprofv3 kernel trace of the bench (steady state) and its median step timeline.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/${TAG:-timeline}
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --steps 50 --warmup 5 --sustain 300 --no-cpu-baseline ${BENCH_ARGS} > "$OUT/bench.log" 2>&1 || exit $?
tail -1 "$OUT/bench.log" | cut -c1-300
f=$(find "$OUT/trace" -name '*kernel_trace.csv' | head -1)
python3 tools/timeline.py "$f" 0.5 0.95 | tee "$OUT/timeline.txt"

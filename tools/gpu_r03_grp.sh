#!/bin/bash
# Grouped layer-1 dW slabs: exactness, rocprof kernel stats, A/B against the
# slab sum over all slabs (GS_DW_NOGROUP=1).
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r03grp
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || exit $?
head -12 "$OUT/prof/run_kernel_stats.csv" | cut -c1-60,200-
ROUNDS=${ROUNDS:-4} bash tools/ab_env_n.sh "GS_X=0" "GS_DW_NOGROUP=1" > "$OUT/ab.txt" 2>&1 || exit $?
tail -3 "$OUT/ab.txt"

#!/bin/bash
# 48-row layer-1 forward tiles: exactness, rocprof stats, A/B against 32-row tiles.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r03rows
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py tests/test_gpu_model.py > "$OUT/tests.log" 2>&1
rc=$?; tail -2 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || exit $?
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')):
    print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,2), round(float(r['MinNs'])/1e3,2))
" | head -11
ROUNDS=4 bash tools/ab_env_k.sh GS_X=0 GS_FWD_ROWS=32 > "$OUT/ab.txt" 2>&1 || exit $?
tail -2 "$OUT/ab.txt"

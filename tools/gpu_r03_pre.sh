#!/bin/bash
# Slab sums and the SGD's norm fold with every load of a round issued before
# the adds: model + full-size tests, rocprof stats, A/B against the previous
# build (libgraphsage_amd_alt.so).
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r03pre
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py tests/test_gpu_model.py tests/test_gpu_dp.py > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || exit $?
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')):
    print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,2), round(float(r['MinNs'])/1e3,2))
"
bash tools/ab_so.sh > "$OUT/ab.txt" 2>&1 || exit $?
cat "$OUT/ab.txt"

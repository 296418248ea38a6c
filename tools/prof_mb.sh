#!/bin/bash
# rocprofv3 kernel trace of the linear microbenchmark; prints per-kernel averages.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/prof_mb_${TAG:-x}
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- \
    python3 ${MB:-tools/mb_linear.py} ${MB_ARGS} > "$OUT/mb.log" 2>&1 || exit $?
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:80]:80s} {int(r['Calls']):6d} avg {float(r['AverageNs'])/1e3:8.2f}us min {float(r['MinNs'])/1e3:8.2f}us")
PY

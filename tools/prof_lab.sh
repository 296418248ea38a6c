#!/bin/bash
# rocprofv3 kernel stats of one lab script: tools/prof_lab.sh TAG script.py [args]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 "$@" > $OUT/log.txt 2>&1
rc=$?
tail -3 $OUT/log.txt
python3 - "$OUT/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:24]:
    print(f"{r['Name'][:70]:70s} n {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:8.1f} {float(r['Percentage']):5.1f}%")
PY
exit $rc

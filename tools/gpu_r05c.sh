#!/bin/bash
# Round-5 pass C: top-launch lab (v1 vs v2 timing + error vs a CPU
# reference), the -m gpu suite on the current build, the default bench line
# and a rocprofv3 kernel-stats pass of the 300-step bench.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r05c
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 120 tools/bin/top_lab tids > "$OUT/top_lab.txt" 2>&1; rc=$?
cat "$OUT/top_lab.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf -s -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/gpu_tests.log"; grep -a "max |emb diff|" "$OUT/gpu_tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || exit $?
python3 - "$OUT/bench_default.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("value", d["value"], "ms", d["ms_per_step"], "sustained", d["sustained"]["value"], d["sustained"]["ms_per_step"], "frac", r["frac"], "frac_live", r["frac_live"], "sampler", d["config"]["sampler"]["ms_per_batch"])
PY
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --ref-stream-steps 0 > "$OUT/prof.log" 2>&1 || exit $?
cp "$OUT/prof/run_kernel_stats.csv" "$OUT/kernel_stats_rmat2m_steps300.csv" && rm -rf "$OUT/prof"
python3 - "$OUT/kernel_stats_rmat2m_steps300.csv" <<'PY'
import csv, sys
for row in csv.DictReader(open(sys.argv[1])):
    if int(row["Calls"]) > 100:
        print(f'{row["Name"][:70]:70s} {row["Calls"]:>5} avg {float(row["AverageNs"])/1e3:6.2f} min {float(row["MinNs"])/1e3:6.2f}')
PY
exit $rc

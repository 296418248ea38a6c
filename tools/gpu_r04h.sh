#!/bin/bash
# Round-4 pass H: the deferred update with the fold after the forward's K loop
# (GPU tests; three alternating bench A/B rounds, GS_DEFER_SGD=0/1), and the
# pack slots on transparent huge pages (GS_PIN_THP=1: runner test, pull
# kernel time under rocprofv3 --stats, bench A/B).
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04h
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_model.py -k "deferred or runner_matches or dw_plus" > "$OUT/gpu_tests.log" 2>&1 \
    || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
GS_PIN_THP=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_model.py -k "runner_matches" > "$OUT/gpu_tests_thp.log" 2>&1 \
    || { tail -30 "$OUT/gpu_tests_thp.log"; exit 1; }
tail -1 "$OUT/gpu_tests_thp.log"
summ() {
python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]
print(sys.argv[2], "value", d["value"], "ms", d["ms_per_step"], "sampler ms", c["sampler"]["ms_per_batch"],
      "sustained", d["sustained"]["value"], d["sustained"]["ms_per_step"], "fwd TF", d["roofline"].get("achieved"))
PY
}
for i in 1 2 3; do
  for C in "0 0" "1 0" "1 1"; do
    set -- $C
    GS_DEFER_SGD=$1 GS_PIN_THP=$2 timeout -k 10 300 python3 bench.py --no-cpu-baseline --ref-stream-steps 0 \
        > "$OUT/bench_d$1_t$2_$i.json" 2> "$OUT/bench_d$1_t$2_$i.err" || exit $?
    summ "$OUT/bench_d$1_t$2_$i.json" "defer $1 thp $2" || exit $?
  done
done
for T in 0 1; do
  GS_PIN_THP=$T timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_t$T" -o run --output-format csv -- python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline --ref-stream-steps 0 --sustain 0 > "$OUT/prof_t$T.log" 2>&1 || exit $?
  cp "$OUT/prof_t$T/run_kernel_stats.csv" "$OUT/kernel_stats_t$T.csv" && rm -rf "$OUT/prof_t$T"
  python3 - "$OUT/kernel_stats_t$T.csv" "thp $T" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(sys.argv[2], r["Name"][:40], "%.2f" % (float(r["AverageNs"]) / 1e3), "min %.2f" % (float(r["MinNs"]) / 1e3))
PY
done

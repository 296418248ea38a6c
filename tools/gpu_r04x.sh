#!/bin/bash
# Round-4 pass X: the layer-2 backward's transposed gather from per-source
# records (GS_TREC): bitwise A/B tests, the model / full-size suites, then a
# bench A/B (GS_TREC=0 / default, fp32, three alternating rounds).
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04x
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_model.py \
    tests/test_gpu_fullsize.py > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
for i in 1 2 3; do
  for TR in 0 1; do
    GS_TREC=$TR timeout -k 10 300 python3 bench.py --no-cpu-baseline --ref-stream-steps 0 --steps 100 \
        > "$OUT/bench_t${TR}_$i.json" 2> "$OUT/bench_t${TR}_$i.err" || exit $?
    python3 - "$OUT/bench_t${TR}_$i.json" "trec $TR" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline_kernels"]
print(sys.argv[2], "value", d["value"], "ms", d["ms_per_step"], "sustained", d["sustained"]["value"],
      d["sustained"]["ms_per_step"], "fwd", k["fwd"]["avg_launch_us"], "dw", k["dw"]["avg_launch_us"], "top", k["top"]["avg_launch_us"])
PY
  done
done
GS_TREC=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/p0" -o run --output-format csv -- python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline --ref-stream-steps 0 --sustain 0 > "$OUT/p0.log" 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/p1" -o run --output-format csv -- python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline --ref-stream-steps 0 --sustain 0 > "$OUT/p1.log" 2>&1 || exit $?
for P in p0 p1; do
  echo "== $P"
  python3 - "$OUT/$P/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "gs::" in r["Name"] and int(r["Calls"]) > 100:
        print(f"  {r['Name'].split('(')[0][-50:]:50s} avg {float(r['AverageNs'])/1e3:7.2f} min {float(r['MinNs'])/1e3:7.2f}")
PY
done
rm -rf "$OUT/p0" "$OUT/p1"

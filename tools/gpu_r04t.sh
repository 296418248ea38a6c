#!/bin/bash
# Round-4 pass T: GS_SELF_ROWS (the side-stream gather also writes the layer-1
# rows' own features; the layer-1 forward and dW read [self | agg] densely):
# the bitwise A/B test, the runner / full-size suites with it on, then bench
# A/B (fp32 MEAN and bf16 MAX, three alternating rounds) and a kernel-stats pass.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04t
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_model.py \
    -k "self_rows" > "$OUT/gpu_tests_ab.log" 2>&1 || { tail -30 "$OUT/gpu_tests_ab.log"; exit 1; }
tail -1 "$OUT/gpu_tests_ab.log"
GS_SELF_ROWS=1 timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_model.py tests/test_gpu_fullsize.py tests/test_gpu_dp.py -k "runner or fullsize or embed or deferred or allreduce" \
    > "$OUT/gpu_tests_on.log" 2>&1 || { tail -30 "$OUT/gpu_tests_on.log"; exit 1; }
tail -1 "$OUT/gpu_tests_on.log"
for i in 1 2 3; do
  for C in rmat2m rmat2m-max-bf16; do
    for SR in 0 1; do
      GS_SELF_ROWS=$SR timeout -k 10 300 python3 bench.py --config $C --no-cpu-baseline --ref-stream-steps 0 \
          > "$OUT/bench_${C}_sr${SR}_$i.json" 2> "$OUT/bench_${C}_sr${SR}_$i.err" || exit $?
      python3 - "$OUT/bench_${C}_sr${SR}_$i.json" "$C self_rows $SR" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline_kernels"]
print(sys.argv[2], "value", d["value"], "ms", d["ms_per_step"], "sustained", d["sustained"]["value"],
      d["sustained"]["ms_per_step"], "fwd", k["fwd"]["avg_launch_us"], "dw", k["dw"]["avg_launch_us"],
      "gather", k["gather"]["avg_launch_us"], "top", k["top"]["avg_launch_us"])
PY
    done
  done
done
GS_SELF_ROWS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --ref-stream-steps 0 > "$OUT/prof.log" 2>&1 || exit $?
cp "$OUT/prof/run_kernel_stats.csv" "$OUT/kernel_stats_rmat2m_self_rows_steps300.csv" && rm -rf "$OUT/prof"
python3 - "$OUT/kernel_stats_rmat2m_self_rows_steps300.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "gs::" in r["Name"] and int(r["Calls"]) > 100:
        print(f"  {r['Name'].split('(')[0][-50:]:50s} avg {float(r['AverageNs'])/1e3:7.2f} min {float(r['MinNs'])/1e3:7.2f}")
PY

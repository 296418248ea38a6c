#!/bin/bash
# Round-4 pass G: the deferred clip + SGD (GPU tests, bench A/B), the top
# launch's head operands staged by the DMA waves (lab A/B), the shared helper
# pool (sampler bench and bench A/B), a kernel trace of the step and the
# gradient-norm probe.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04g
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_model.py tests/test_gpu_fullsize.py -k "deferred or runner or top_launch or fused_backward or dw_plus" \
    > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
for i in 1 2; do
  for V in base stage; do
    for M in plain tids; do
      echo "== $V $M round $i" >> "$OUT/top_lab_ab.txt"
      timeout -k 10 60 tools/bin/top_lab_$V $M >> "$OUT/top_lab_ab.txt" 2>&1 || exit $?
    done
  done
done
grep -A1 "==" "$OUT/top_lab_ab.txt" | grep -v "^--"
for i in 1 2; do
  for C in "0 0 0" "1 0 0" "1 1 0" "1 0 1"; do
    set -- $C
    GS_DEFER_SGD=$1 GS_SHARED_HELPERS=$2 GS_DW_PLUS=$3 timeout -k 10 300 python3 bench.py --no-cpu-baseline \
        --ref-stream-steps 0 > "$OUT/bench_d$1_s$2_p$3_$i.json" 2> "$OUT/bench_d$1_s$2_p$3_$i.err" || exit $?
    python3 - "$OUT/bench_d$1_s$2_p$3_$i.json" "defer $1 shared $2 dwplus $3" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]
print(sys.argv[2], "value", d["value"], "ms", d["ms_per_step"], "sampler ms", c["sampler"]["ms_per_batch"],
      "sustained", d["sustained"]["value"], d["sustained"]["ms_per_step"])
PY
  done
done
for i in 1 2; do
  timeout -k 10 200 tools/bin/sampler_bench_pool 1 200 7 0 >> "$OUT/sampler_ab.txt" 2>&1 || exit $?
  timeout -k 10 200 tools/bin/sampler_bench_pool 1 200 7 1 >> "$OUT/sampler_ab.txt" 2>&1 || exit $?
done
grep helpers "$OUT/sampler_ab.txt"
# kernel trace of a short default bench: the step's timeline (main / side overlap)
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- python3 bench.py --steps 60 --warmup 5 --no-cpu-baseline --sustain 0 --ref-stream-steps 0 > "$OUT/trace.log" 2>&1 || exit $?
cp "$OUT/trace/run_kernel_trace.csv" "$OUT/kernel_trace.csv" && rm -rf "$OUT/trace"
echo trace ok
timeout -k 10 300 python3 tools/norm_probe.py rmat2m 300 > "$OUT/norm_probe.txt" 2>&1 || exit $?
tail -1 "$OUT/norm_probe.txt"

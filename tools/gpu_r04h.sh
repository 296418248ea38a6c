#!/bin/bash
# Round-4 pass H: the deferred update with its parameter update spread over
# the forward's workgroups: GPU tests, three alternating bench A/B rounds
# (GS_DEFER_SGD=0/1), rocprofv3 kernel stats of the 300-step bench with the
# deferred update, and the gradient-norm probe (how often the clip scales).
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04h
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_model.py -k "deferred or runner_matches or dw_plus" > "$OUT/gpu_tests.log" 2>&1 \
    || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
for i in 1 2 3; do
  for D in 0 1; do
    GS_DEFER_SGD=$D timeout -k 10 300 python3 bench.py --no-cpu-baseline --ref-stream-steps 0 \
        > "$OUT/bench_d${D}_$i.json" 2> "$OUT/bench_d${D}_$i.err" || exit $?
    python3 - "$OUT/bench_d${D}_$i.json" "defer $D" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]
print(sys.argv[2], "value", d["value"], "ms", d["ms_per_step"], "sampler ms", c["sampler"]["ms_per_batch"],
      "sustained", d["sustained"]["value"], d["sustained"]["ms_per_step"], "fwd us", d["roofline"].get("achieved"))
PY
  done
done
: timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --ref-stream-steps 0 > "$OUT/prof.log" 2>&1 || exit $?
: cp "$OUT/kernel_stats_rmat2m_steps300.csv" && rm -rf "$OUT/prof"
: head -12 "$OUT/kernel_stats_rmat2m_steps300.csv" | cut -c1-160
: timeout -k 10 300 python3 tools/norm_probe.py rmat2m 300 > "$OUT/norm_probe.txt" 2>&1 || exit $?
: tail -1

#!/bin/bash
# Round-4 pass L: the deferred update on the all-reduce path: model / DP /
# full-size GPU tests, one default bench line.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04l
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_model.py tests/test_gpu_dp.py tests/test_gpu_fullsize.py > "$OUT/gpu_tests.log" 2>&1 \
    || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("value", d["value"], "ms", d["ms_per_step"], "sustained", d["sustained"]["value"], "| roofline", r["avg_launch_us"], r["frac"], r["timer"][:12])
PY

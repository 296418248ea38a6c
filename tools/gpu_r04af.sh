#!/bin/bash
# Round-4 pass AF: the top launch on 8 waves (default) — the model / full-size /
# DP GPU suites, then bench A/B against GS_TOP_E8=0 (fp32 MEAN and bf16 MAX,
# three alternating rounds).
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04af
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_model.py \
    tests/test_gpu_fullsize.py tests/test_gpu_dp.py tests/test_gpu_pubmed.py > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
for i in 1 2 3; do
  for C in rmat2m rmat2m-max-bf16; do
    for E in 0 1; do
      GS_TOP_E8=$E timeout -k 10 300 python3 bench.py --config $C --no-cpu-baseline --ref-stream-steps 0 --steps 100 \
          > "$OUT/bench_${C}_e${E}_$i.json" 2> "$OUT/bench_${C}_e${E}_$i.err" || exit $?
      python3 - "$OUT/bench_${C}_e${E}_$i.json" "$C e8 $E" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline_kernels"]
print(sys.argv[2], "value", d["value"], "ms", d["ms_per_step"], "sustained", d["sustained"]["value"],
      d["sustained"]["ms_per_step"], "top", k["top"]["avg_launch_us"], "fwd", k["fwd"]["avg_launch_us"])
PY
    done
  done
done

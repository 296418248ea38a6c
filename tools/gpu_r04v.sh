#!/bin/bash
# Round-4 pass V: forward row tiles re-checked with the dense [self | agg] slot
# (GS_FWD_ROWS=32 against 48 at rmat2m; 48 was then the default), three alternating rounds.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04v
mkdir -p "$OUT"; cd "$ROOT"
for i in 1 2 3; do
  for R in 48 32; do
    GS_FWD_ROWS=$R timeout -k 10 300 python3 bench.py --no-cpu-baseline --ref-stream-steps 0 --steps 100 \
        > "$OUT/bench_r${R}_$i.json" 2> "$OUT/bench_r${R}_$i.err" || exit $?
    python3 - "$OUT/bench_r${R}_$i.json" "rows $R" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline_kernels"]
print(sys.argv[2], "value", d["value"], "ms", d["ms_per_step"], "sustained", d["sustained"]["value"],
      d["sustained"]["ms_per_step"], "fwd", k["fwd"]["avg_launch_us"], k["fwd"]["kernel"][-28:], "dw", k["dw"]["avg_launch_us"])
PY
  done
done

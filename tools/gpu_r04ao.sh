#!/bin/bash
# Round-4 pass AO: forward row tiles for bf16 MAX (GS_FWD_ROWS=48 against the
# default 32), the driver's default command and a 300-step run, alternating.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04ao
mkdir -p "$OUT"; cd "$ROOT"
for i in 1 2 3; do
  for R in 48 32; do
    for K in 20 100; do
      GS_FWD_ROWS=$R timeout -k 10 300 python3 bench.py --config rmat2m-max-bf16 --no-cpu-baseline --ref-stream-steps 0 --steps $K \
          > "$OUT/bench_r${R}_k${K}_$i.json" 2> "$OUT/bench_r${R}_k${K}_$i.err" || exit $?
      python3 - "$OUT/bench_r${R}_k${K}_$i.json" "rows $R steps $K" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline_kernels"]
print(sys.argv[2], "value", d["value"], "ms", d["ms_per_step"], "sustained", d["sustained"]["value"],
      d["sustained"]["ms_per_step"], "fwd", k["fwd"]["avg_launch_us"], "dw", k["dw"]["avg_launch_us"])
PY
    done
  done
done

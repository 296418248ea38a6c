#!/bin/bash
# Round-4 pass AP: side-stream gating re-checked with the
# dense [self | agg] slot (GS_SIDE_GATE_STEP, GS_RUNNER_GATE_FWD) with the final step, three alternating rounds.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04ap
mkdir -p "$OUT"; cd "$ROOT"
for i in 1 2 3; do
  for V in default sidegate gatefwd; do
    case $V in
      default) E="" ;;
      sidegate) E="GS_SIDE_GATE_STEP=1" ;;
      gatefwd) E="GS_RUNNER_GATE_FWD=1" ;;
    esac
    env $E timeout -k 10 300 python3 bench.py --no-cpu-baseline --ref-stream-steps 0 --steps 100 \
        > "$OUT/bench_${V}_$i.json" 2> "$OUT/bench_${V}_$i.err" || exit $?
    python3 - "$OUT/bench_${V}_$i.json" "$V" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["roofline_kernels"]
print(sys.argv[2], "value", d["value"], "ms", d["ms_per_step"], "sustained", d["sustained"]["value"],
      d["sustained"]["ms_per_step"], "fwd", k["fwd"]["avg_launch_us"], "dw", k["dw"]["avg_launch_us"])
PY
  done
done

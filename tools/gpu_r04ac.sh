#!/bin/bash
# Round-4 pass AC: the pack pull placement and the gather grid re-checked with the
# dense [self | agg] slot (GS_PULL_COPY, GS_PULL_AHEAD, GS_AGG_BLOCKS), three alternating rounds.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04ac
mkdir -p "$OUT"; cd "$ROOT"
for i in 1 2 3; do
  for V in default pullcopy pullahead aggblocks; do
    case $V in
      default) E="" ;;
      pullcopy) E="GS_PULL_COPY=1" ;;
      pullahead) E="GS_PULL_AHEAD=1" ;;
      aggblocks) E="GS_AGG_BLOCKS=256" ;;
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

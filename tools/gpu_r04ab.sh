#!/bin/bash
# Round-4 pass AB: the layer-1 dW grid and the dW-plus layout re-checked with the
# dense [self | agg] slot (GS_DW_BLOCKS, GS_DW_PLUS), three alternating rounds.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04ab
mkdir -p "$OUT"; cd "$ROOT"
for i in 1 2 3; do
  for V in default blocks256 blocks768 blocks1024 dwplus; do
    case $V in
      default) E="" ;;
      blocks256) E="GS_DW_BLOCKS=256" ;;
      blocks768) E="GS_DW_BLOCKS=768" ;;
      blocks1024) E="GS_DW_BLOCKS=1024" ;;
      dwplus) E="GS_DW_PLUS=1" ;;
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

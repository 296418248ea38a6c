#!/bin/bash
# Round-4 pass AJ: GS_RUNNER_YIELD (the runner's completion poll yields its core
# every 64 polls) against the default spin, the driver's default command
# (20 steps + the 200-step sustained window), four alternating rounds.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04aj
mkdir -p "$OUT"; cd "$ROOT"
for i in 1 2 3 4; do
  for Y in 0 1; do
    GS_RUNNER_YIELD=$Y timeout -k 10 300 python3 bench.py --no-cpu-baseline > "$OUT/bench_y${Y}_$i.json" 2> "$OUT/bench_y${Y}_$i.err" || exit $?
    python3 - "$OUT/bench_y${Y}_$i.json" "yield $Y" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d["sustained"]
print(sys.argv[2], "value", d["value"], "sampler", d["config"]["sampler"]["ms_per_batch"], "sustained", s["value"],
      "sus sampler", s["host_ms_per_step"]["sample"], "misses", s["lookahead_misses"], "ref", d["reference_stream"]["value"])
PY
  done
done

#!/bin/bash
# Round-4 pass AM: sampler layouts re-checked with the final step (streams x
# helpers per stream: 7x1 default, 8x1, 12x0), the driver's default command,
# three alternating rounds.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04am
mkdir -p "$OUT"; cd "$ROOT"
for i in 1 2 3; do
  for L in 7:1 8:1 12:0; do
    S=${L%%:*}; H=${L##*:}
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --ref-stream-steps 0 --sampler-streams $S --sampler-helpers $H \
        > "$OUT/bench_s${S}_h${H}_$i.json" 2> "$OUT/bench_s${S}_h${H}_$i.err" || exit $?
    python3 - "$OUT/bench_s${S}_h${H}_$i.json" "layout $L" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d["sustained"]
print(sys.argv[2], "value", d["value"], "sampler", d["config"]["sampler"]["ms_per_batch"], "sustained", s["value"],
      "sus sampler", s["host_ms_per_step"]["sample"], "misses", s["lookahead_misses"])
PY
  done
done

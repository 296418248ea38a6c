#!/bin/bash
# Round-4 pass M: side-stream placement on the deferred step (GS_SIDE_GATE_STEP,
# GS_RUNNER_GATE_FWD) and 6 sampler streams, alternating, three rounds.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04m
mkdir -p "$OUT"; cd "$ROOT"
for i in 1 2 3; do
  for V in default gate_step gate_fwd s6; do
    unset GS_SIDE_GATE_STEP GS_RUNNER_GATE_FWD; EXTRA=""
    case $V in
      gate_step) export GS_SIDE_GATE_STEP=1 ;;
      gate_fwd) export GS_RUNNER_GATE_FWD=1 ;;
      s6) EXTRA="--sampler-streams 6" ;;
    esac
    timeout -k 10 400 python3 bench.py --no-cpu-baseline --ref-stream-steps 0 $EXTRA > "$OUT/bench_${V}_$i.json" 2> "$OUT/bench_${V}_$i.err" || exit $?
    echo -n "$V "
    python3 - "$OUT/bench_${V}_$i.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"], "sampler ms", d["config"]["sampler"]["ms_per_batch"],
      "sustained", d["sustained"]["value"], d["sustained"]["ms_per_step"], "misses", d["sustained"]["lookahead_misses"])
PY
  done
done
unset GS_SIDE_GATE_STEP GS_RUNNER_GATE_FWD

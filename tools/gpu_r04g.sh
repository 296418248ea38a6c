#!/bin/bash
# Round-4 pass G: shared helper pool A/B.  The sampler bench (7 streams,
# private helpers vs one shared pool, same thread count) and the default
# bench with GS_SHARED_HELPERS=0/1, twice each, alternating.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04g
mkdir -p "$OUT"; cd "$ROOT"
for i in 1 2; do
  timeout -k 10 200 tools/bin/sampler_bench_pool 1 200 7 0 >> "$OUT/sampler_ab.txt" 2>&1 || exit $?
  timeout -k 10 200 tools/bin/sampler_bench_pool 1 200 7 1 >> "$OUT/sampler_ab.txt" 2>&1 || exit $?
done
grep helpers "$OUT/sampler_ab.txt"
for i in 1 2; do
  for S in 0 1; do
    GS_SHARED_HELPERS=$S timeout -k 10 300 python3 bench.py --no-cpu-baseline --ref-stream-steps 0 > "$OUT/bench_s${S}_$i.json" 2> "$OUT/bench_s${S}_$i.err" || exit $?
    python3 - "$OUT/bench_s${S}_$i.json" $S <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]
print("shared", sys.argv[2], "value", d["value"], "ms", d["ms_per_step"], "sampler ms", c["sampler"]["ms_per_batch"],
      "sustained", d["sustained"]["value"], d["sustained"]["ms_per_step"])
PY
  done
done

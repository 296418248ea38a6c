#!/bin/bash
# Round-4 pass Q: the last hop's draws in two passes (the stream's thread draws,
# helpers finish chunks: pool swaps, row offsets, dst ids) and the threshold
# compare of the pool window, the frontier row_ptr prefetched under the union merge, against the previous sampler (sampler bench,
# alternating binaries), then the bench line on the two-pass library.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04q
mkdir -p "$OUT"; cd "$ROOT"
for i in 1 2; do
  for cfg in "1 200 1" "7 200 1" "1 200 7"; do
    for V in base 2pass 2pass_thr 2pass_pf; do
      echo "== $V [$cfg] round $i" >> "$OUT/sampler_ab.txt"
      timeout -k 10 200 tools/bin/sampler_bench_$V $cfg >> "$OUT/sampler_ab.txt" 2>&1 || exit $?
    done
  done
done
grep -E "==|helpers" "$OUT/sampler_ab.txt"
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]
print("value", d["value"], "ms", d["ms_per_step"], "sampler ms", c["sampler"]["ms_per_batch"], "sustained",
      d["sustained"]["value"], d["sustained"]["ms_per_step"], "misses", d["sustained"]["lookahead_misses"],
      "ref", d["reference_stream"]["value"], d["reference_stream"]["sampler"])
PY

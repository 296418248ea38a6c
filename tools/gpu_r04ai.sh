#!/bin/bash
# Round-4 pass AI (and AL, after the runner yield): the final build once more — the whole GPU suite, smoke(),
# and the driver's default bench command.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04al
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
    > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 500 python3 bench.py > "$OUT/bench_rmat2m.json" 2> "$OUT/bench_rmat2m.err" || exit $?
python3 - "$OUT/bench_rmat2m.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]; r = d["roofline"]
print("value", d["value"], "ms", d["ms_per_step"], "sampler ms", c["sampler"]["ms_per_batch"], "sustained",
      d["sustained"]["value"], "misses", d["sustained"]["lookahead_misses"], "roofline", r["kernel"][:44], r["achieved"],
      r["frac"], "rocprof", (r.get("rocprof") or {}).get("avg_us"), "cpu", d["cpu_baseline"]["value"], "ref",
      d["reference_stream"]["value"])
PY

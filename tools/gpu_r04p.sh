#!/bin/bash
# Round-4 pass P: final validation of the defaults (deferred update incl. after the all-reduce,
# KStamp timer, THP pack slots; fp32 and bf16): the whole GPU suite, smoke(), bench lines
# alternating rmat2m / rmat2m-max-bf16.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04p
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
    > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
for i in 1 2 3 4; do
  C=rmat2m; [ $((i % 2)) -eq 0 ] && C=rmat2m-max-bf16
  timeout -k 10 400 python3 bench.py --config $C > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err" || exit $?
  echo -n "$C "
  python3 - "$OUT/bench_$i.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]; r = d["roofline"]
print("value", d["value"], "ms", d["ms_per_step"], "sampler ms", c["sampler"]["ms_per_batch"], "sustained",
      d["sustained"]["value"], d["sustained"]["ms_per_step"], "misses", d["sustained"]["lookahead_misses"],
      "roofline", r["kernel"][:40], r["achieved"], r["unit"], r["frac"], "ref", (d.get("reference_stream") or {}).get("value"))
PY
done

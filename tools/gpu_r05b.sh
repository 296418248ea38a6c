#!/bin/bash
# Round-5 pass B: the -m gpu suite on the pruned build (with the new
# full-size timed-step parity tests), then the default bench line.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r05b
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf -s -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/gpu_tests.log"; grep -a "max |emb diff|" "$OUT/gpu_tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || exit $?
python3 - "$OUT/bench_default.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("value", d["value"], "ms", d["ms_per_step"], "sustained", d["sustained"]["value"], "frac", r["frac"], "frac_live", r["frac_live"], "traffic", r["traffic"], r.get("traffic_dispatches"))
PY
exit $rc

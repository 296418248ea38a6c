#!/bin/bash
# Round-4 pass K: the roofline timers on the kernels' own spans (KStamp) for
# the forward and top launches: the timer tests, bench lines fp32 / bf16.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04k
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_model.py -k "timer or deferred_update_switch" > "$OUT/gpu_tests.log" 2>&1 \
    || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
for C in rmat2m rmat2m-max-bf16 rmat2m; do
  timeout -k 10 400 python3 bench.py --config $C > "$OUT/bench_$C.json" 2> "$OUT/bench_$C.err" || exit $?
  echo -n "$C "
  python3 - "$OUT/bench_$C.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]; r = d["roofline"]
print("value", d["value"], "ms", d["ms_per_step"], "sustained", d["sustained"]["value"], d["sustained"]["ms_per_step"],
      "| roofline", r["kernel"][:44], r["avg_launch_us"], "us", r["achieved"], r["unit"], r["frac"], "rocprof", r.get("rocprof"))
for k, v in d.get("roofline_kernels", {}).items():
    print("   ", k, v.get("avg_launch_us"), v.get("achieved"), v.get("frac"), (v.get("rocprof") or {}).get("avg_us"))
PY
done
# the pack pull on the copy engine (GS_PULL_COPY=1) against the pull kernel, with the deferred step
for i in 1 2; do
  for P in 0 1; do
    if [ $P -eq 1 ]; then export GS_PULL_COPY=1; else unset GS_PULL_COPY; fi
    timeout -k 10 400 python3 bench.py --no-cpu-baseline --ref-stream-steps 0 > "$OUT/bench_pc${P}_$i.json" 2> "$OUT/bench_pc${P}_$i.err" || exit $?
    echo -n "pull_copy $P "
    python3 - "$OUT/bench_pc${P}_$i.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"], "sustained", d["sustained"]["value"], d["sustained"]["ms_per_step"])
PY
  done
done
unset GS_PULL_COPY

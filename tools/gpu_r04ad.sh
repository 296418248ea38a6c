#!/bin/bash
# Round-4 pass AD: the driver's default bench command on the final build
# (fp32 MEAN, then bf16 MAX), with the CPU baseline and the reference stream.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04ad
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 500 python3 bench.py > "$OUT/bench_rmat2m.json" 2> "$OUT/bench_rmat2m.err" || exit $?
timeout -k 10 500 python3 bench.py --config rmat2m-max-bf16 > "$OUT/bench_rmat2m_max_bf16.json" 2> "$OUT/bench_bf16.err" || exit $?
for f in bench_rmat2m bench_rmat2m_max_bf16; do
python3 - "$OUT/$f.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]; r = d["roofline"]
print(sys.argv[1].split("/")[-1], "value", d["value"], "ms", d["ms_per_step"], "sampler ms", c["sampler"]["ms_per_batch"],
      "sustained", d["sustained"]["value"], "misses", d["sustained"]["lookahead_misses"],
      "roofline", r["kernel"][:44], r["achieved"], r["unit"], r["frac"], "rocprof", (r.get("rocprof") or {}).get("avg_us"),
      "cpu", d["cpu_baseline"]["value"], "ref", d["reference_stream"]["value"])
for k, v in d["roofline_kernels"].items():
    print("   ", k, v["achieved"], v["unit"], v["frac"], v["avg_launch_us"], (v.get("rocprof") or {}).get("avg_us"), v.get("traffic"), v.get("mfma_busy"))
PY
done

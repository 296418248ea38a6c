#!/bin/bash
# Round-4 pass AN: the final build on the rmat16m workload (the per-GPU share of
# the 8-GPU config: scale 24, 160 M pairs, F = 128) and 300-step fp32 / bf16 lines.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04an
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 900 python3 -u bench.py --config rmat16m --steps 100 --no-cpu-baseline > "$OUT/bench_rmat16m.json" 2> "$OUT/bench_rmat16m.err" || { tail -5 "$OUT/bench_rmat16m.err"; exit 1; }
timeout -k 10 400 python3 bench.py --steps 300 --warmup 5 --sustain 300 --no-cpu-baseline > "$OUT/bench_rmat2m_steps300.json" 2> "$OUT/b2.err" || exit $?
timeout -k 10 400 python3 bench.py --config rmat2m-max-bf16 --steps 300 --warmup 5 --sustain 300 --no-cpu-baseline > "$OUT/bench_rmat2m_max_bf16_steps300.json" 2> "$OUT/b3.err" || exit $?
for f in bench_rmat16m bench_rmat2m_steps300 bench_rmat2m_max_bf16_steps300; do
python3 - "$OUT/$f.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split("/")[-1], "value", d["value"], "ms", d["ms_per_step"], "sustained", (d.get("sustained") or {}).get("value"),
      "sampler", d["config"]["sampler"]["ms_per_batch"], "roofline", d["roofline"]["kernel"][:40], d["roofline"]["frac"])
PY
done

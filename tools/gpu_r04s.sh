#!/bin/bash
# Round-4 pass S: PMC passes (HBM traffic, MFMA busy) for the bf16 MAX config,
# then the default bench line (its roofline entries now carry mfma_busy).
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04s
mkdir -p "$OUT/pmc" "$OUT/mfma"; cd "$ROOT"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $C -d "$OUT/pmc/$C" -o run --output-format csv -- \
      python3 bench.py --config rmat2m-max-bf16 --steps 30 --warmup 5 --no-cpu-baseline --sustain 0 --ref-stream-steps 0 > "$OUT/pmc/bench_$C.log" 2>&1 || exit $?
done
python3 tools/pmc_summary.py "$OUT/pmc" rmat2m-max-bf16 > "$OUT/pmc_traffic_rmat2m_max_bf16.json" || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE \
    -d "$OUT/mfma/pmc" -o run --output-format csv -- \
    python3 bench.py --config rmat2m-max-bf16 --steps 30 --warmup 5 --sustain 0 --no-cpu-baseline --ref-stream-steps 0 > "$OUT/mfma/bench.log" 2>&1 || exit $?
python3 tools/pmc_mfma_summary.py "$OUT/mfma" > "$OUT/pmc_mfma_rmat2m_max_bf16.json" || exit $?
rm -rf "$OUT/pmc/FETCH_SIZE" "$OUT/pmc/WRITE_SIZE" "$OUT/mfma/pmc"
echo pmc ok
cp "$OUT/pmc_traffic_rmat2m_max_bf16.json" "$OUT/pmc_mfma_rmat2m_max_bf16.json" profiles/ 2>/dev/null
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
timeout -k 10 400 python3 bench.py --config rmat2m-max-bf16 --no-cpu-baseline > "$OUT/bench_bf16.json" 2> "$OUT/bench_bf16.err" || exit $?
for f in bench bench_bf16; do
python3 - "$OUT/$f.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[1].split("/")[-1], "value", d["value"], "sustained", d["sustained"]["value"], "roofline", r["kernel"][:44], r["frac"],
      "mfma_busy", r.get("mfma_busy"), "traffic", r.get("traffic"))
for k, v in d["config"].get("roofline_kernels", {}).items():
    print("  ", k, v.get("frac"), v.get("mfma_busy"), v.get("traffic"))
PY
done

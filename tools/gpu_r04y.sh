#!/bin/bash
# Round-4 pass Y: the rest of pass W (its bf16 PMC summary step had a wrong log path):
# bf16 PMC traffic and MFMA busy, the 300-step lines and the kernel timeline.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04y
mkdir -p "$OUT/pmcb" "$OUT/mfmab"; cd "$ROOT"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $C -d "$OUT/pmcb/$C" -o run --output-format csv -- \
      python3 bench.py --config rmat2m-max-bf16 --steps 30 --warmup 5 --no-cpu-baseline --sustain 0 --ref-stream-steps 0 > "$OUT/pmcb/bench_$C.log" 2>&1 || exit $?
done
python3 tools/pmc_summary.py "$OUT/pmcb" rmat2m-max-bf16 > "$OUT/pmc_traffic_rmat2m_max_bf16.json" || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE \
    -d "$OUT/mfmab/pmc" -o run --output-format csv -- \
    python3 bench.py --config rmat2m-max-bf16 --steps 30 --warmup 5 --sustain 0 --no-cpu-baseline --ref-stream-steps 0 > "$OUT/mfmab/bench.log" 2>&1 || exit $?
python3 tools/pmc_mfma_summary.py "$OUT/mfmab" > "$OUT/pmc_mfma_rmat2m_max_bf16.json" || exit $?
rm -rf "$OUT/pmcb" "$OUT/mfmab/pmc"
echo pmc ok
timeout -k 10 400 python3 bench.py --steps 300 --warmup 5 --sustain 300 > "$OUT/bench_rmat2m_steps300.json" 2> "$OUT/bench_rmat2m_steps300.err" || exit $?
timeout -k 10 400 python3 bench.py --config rmat2m-max-bf16 --steps 300 --warmup 5 --sustain 300 > "$OUT/bench_rmat2m_max_bf16_steps300.json" 2> "$OUT/bench_bf16.err" || exit $?
for f in bench_rmat2m_steps300 bench_rmat2m_max_bf16_steps300; do
python3 - "$OUT/$f.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]
print(sys.argv[1].split("/")[-1], "value", d["value"], "ms", d["ms_per_step"], "sampler ms", c["sampler"]["ms_per_batch"], "sustained", d["sustained"]["value"], d["sustained"]["ms_per_step"], "ref", (d.get("reference_stream") or {}).get("value"))
PY
done
# kernel trace of a short default bench: the step's timeline (main / side overlap)
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- python3 bench.py --steps 60 --warmup 5 --no-cpu-baseline --sustain 0 --ref-stream-steps 0 > "$OUT/trace.log" 2>&1 || exit $?
cp "$OUT/trace/run_kernel_trace.csv" "$OUT/kernel_trace.csv" && rm -rf "$OUT/trace"
python3 tools/timeline.py "$OUT/kernel_trace.csv" > "$OUT/timeline.txt" 2>&1; cat "$OUT/timeline.txt"

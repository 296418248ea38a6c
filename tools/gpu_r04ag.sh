#!/bin/bash
# Round-4 pass AG: final validation of the round's defaults — the whole GPU
# suite, smoke(), rocprofv3 kernel stats (fp32 / bf16, 300 steps), PMC HBM
# traffic and MFMA busy (fp32), and the driver's default bench command.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04ag
mkdir -p "$OUT/pmc" "$OUT/mfma"; cd "$ROOT"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
    > "$OUT/gpu_tests.log" 2>&1 || { tail -40 "$OUT/gpu_tests.log"; exit 1; }
tail -1 "$OUT/gpu_tests.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_rmat2m" -o run --output-format csv -- python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --ref-stream-steps 0 > "$OUT/prof_rmat2m.log" 2>&1 || exit $?
cp "$OUT/prof_rmat2m/run_kernel_stats.csv" "$OUT/kernel_stats_rmat2m_steps300.csv" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bf16" -o run --output-format csv -- python3 bench.py --config rmat2m-max-bf16 --steps 300 --warmup 5 --no-cpu-baseline --ref-stream-steps 0 > "$OUT/prof_bf16.log" 2>&1 || exit $?
cp "$OUT/prof_bf16/run_kernel_stats.csv" "$OUT/kernel_stats_rmat2m_max_bf16_steps300.csv" || exit 1
rm -rf "$OUT/prof_rmat2m" "$OUT/prof_bf16"
echo stats ok
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $C -d "$OUT/pmc/$C" -o run --output-format csv -- \
      python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --sustain 0 --ref-stream-steps 0 > "$OUT/pmc/bench_$C.log" 2>&1 || exit $?
done
python3 tools/pmc_summary.py "$OUT/pmc" rmat2m > "$OUT/pmc_traffic_rmat2m.json" || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE \
    -d "$OUT/mfma/pmc" -o run --output-format csv -- \
    python3 bench.py --steps 30 --warmup 5 --sustain 0 --no-cpu-baseline --ref-stream-steps 0 > "$OUT/mfma/bench.log" 2>&1 || exit $?
python3 tools/pmc_mfma_summary.py "$OUT/mfma" > "$OUT/pmc_mfma_rmat2m.json" || exit $?
rm -rf "$OUT/pmc/FETCH_SIZE" "$OUT/pmc/WRITE_SIZE" "$OUT/mfma/pmc"
echo pmc ok
timeout -k 10 500 python3 bench.py > "$OUT/bench_rmat2m.json" 2> "$OUT/bench_rmat2m.err" || exit $?
timeout -k 10 500 python3 bench.py --config rmat2m-max-bf16 > "$OUT/bench_rmat2m_max_bf16.json" 2> "$OUT/bench_bf16.err" || exit $?
for f in bench_rmat2m bench_rmat2m_max_bf16; do
python3 - "$OUT/$f.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]; r = d["roofline"]
print(sys.argv[1].split("/")[-1], "value", d["value"], "ms", d["ms_per_step"], "sampler ms", c["sampler"]["ms_per_batch"],
      "sustained", d["sustained"]["value"], "misses", d["sustained"]["lookahead_misses"],
      "roofline", r["kernel"][:44], r["achieved"], r["unit"], r["frac"], "ref", d["reference_stream"]["value"])
PY
done

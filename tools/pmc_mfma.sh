#!/bin/bash
# MFMA utilisation per kernel from one rocprofv3 --pmc pass (SQ and GRBM
# counters only; no trace domains beside --pmc).  Writes
# gpurun_out/pmc_mfma_$TAG/summary.json (tools/pmc_mfma_summary.py).
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/pmc_mfma_${TAG:-x}
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE \
    -d "$OUT/pmc" -o run --output-format csv -- \
    python3 bench.py --steps 30 --warmup 5 --sustain 0 --no-cpu-baseline ${BENCH_ARGS} > "$OUT/bench.log" 2>&1 || exit $?
python3 tools/pmc_mfma_summary.py "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"

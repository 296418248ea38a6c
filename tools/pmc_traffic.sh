#!/bin/bash
# HBM traffic per dispatch from rocprofv3 PMC counters, one counter per pass
# (FETCH_SIZE and WRITE_SIZE cannot share a TCC pass on gfx950), no trace
# domains alongside --pmc.  Writes gpurun_out/pmc_$TAG/summary.json.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/pmc_${TAG:-x}
mkdir -p "$OUT"
cd "$ROOT"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C -d "$OUT/$C" -o run --output-format csv -- \
      python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > "$OUT/bench_$C.log" 2>&1 || exit $?
done
python3 tools/pmc_summary.py "$OUT" "${CONFIG:-rmat2m}" > "$OUT/summary.json" && cat "$OUT/summary.json"

#!/bin/bash
# Round-2 GPU pass (session 4): parity tests, smoke, the driver's bench
# command, a 300-step bench, the pubmed apply_model bench, the bf16 and
# rmat16m lines, and rocprofv3 kernel stats of the 300-step command.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r02c
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread \
    > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/gpu_tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
run() {  # name, args
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err"
  local rc=$?; echo "bench $name rc=$rc"; tail -c 400 "$OUT/bench_$name.json"; echo; return $rc
}
run default --gpus 1 --steps 20 --warmup 5 || exit $?
run steps300 --gpus 1 --steps 300 --warmup 5 --no-cpu-baseline || exit $?
run pubmed --config pubmed --steps 20 --warmup 3 || exit $?
run max_bf16 --config rmat2m-max-bf16 --steps 300 --warmup 5 --no-cpu-baseline || exit $?
run rmat16m --config rmat16m --steps 300 --warmup 5 --no-cpu-baseline || exit $?
run embed --config rmat2m-embed --full-graph --no-cpu-baseline || exit $?
mkdir -p "$OUT/prof"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline > "$OUT/prof/bench.json" 2> "$OUT/prof/bench.err"
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
rm -f "$OUT/prof/run_kernel_trace.csv"
# HBM traffic (FETCH_SIZE / WRITE_SIZE passes) and MFMA utilisation, rmat2m B=512
TAG=r02c CONFIG=rmat2m bash tools/pmc_traffic.sh > "$OUT/pmc_traffic.log" 2>&1
rc=$?; echo "pmc traffic rc=$rc"; [ $rc -eq 0 ] || exit $rc
TAG=r02c bash tools/pmc_mfma.sh > "$OUT/pmc_mfma.log" 2>&1
rc=$?; echo "pmc mfma rc=$rc"; exit $rc

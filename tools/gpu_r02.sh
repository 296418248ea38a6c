#!/bin/bash
# Round-2 GPU pass: parity tests (no -x: report every failure), smoke, the
# driver's bench command, a 300-step bench, rocprofv3 kernel stats.
# Stops at the first crash (abort/segfault/timeout); pytest rc 1 continues.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/${TAG:-r02}
mkdir -p "$OUT"
cd "$ROOT"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread \
      ${TESTS} > "$OUT/gpu_tests.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -25 "$OUT/gpu_tests.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS} > "$OUT/bench_default.log" 2>&1
  rc=$?; echo "bench default rc=$rc"; tail -1 "$OUT/bench_default.log"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python bench.py --gpus 1 --steps 300 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > "$OUT/bench_300.log" 2>&1
  rc=$?; echo "bench 300 rc=$rc"; tail -1 "$OUT/bench_300.log"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$PROF" ]; then
  mkdir -p "$OUT/prof"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
      python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > "$OUT/prof/bench.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -1 "$OUT/prof/bench.log"; exit $rc
fi

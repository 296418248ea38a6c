#!/bin/bash
# GPU-box pass: parity tests, smoke, benches, rocprofv3 kernel trace.
# Stops at the first crash (abort/segfault/timeout); a plain pytest failure (rc 1) continues.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -rf -p no:cacheprovider > "$OUT/gpu_tests.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/gpu_tests.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
fi
for S in ${STREAMS:-1 4}; do
  timeout -k 10 600 python bench.py --steps ${STEPS:-100} --warmup 10 --sampler-streams $S ${BENCH_ARGS} \
      > "$OUT/bench_s$S.log" 2>&1
  rc=$?; echo "bench streams=$S rc=$rc"; tail -1 "$OUT/bench_s$S.log"; [ $rc -eq 0 ] || exit $rc
  BENCH_ARGS="$BENCH_ARGS --no-cpu-baseline"
done
if [ -n "$PROF" ]; then
  mkdir -p "$OUT/prof_$PROF"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$PROF" -o run --output-format csv -- \
      python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --sampler-streams ${PROF_STREAMS:-4} ${PROF_ARGS} \
      > "$OUT/prof_$PROF/bench.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -1 "$OUT/prof_$PROF/bench.log"; exit $rc
fi

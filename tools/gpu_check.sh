#!/bin/bash
# One GPU-box pass: parity tests, smoke, short bench.  Stops at the first crash
# (abort/segfault/timeout); a plain test failure (pytest rc 1) still benches.
set -o pipefail
mkdir -p gpurun_out
STEPS=${STEPS:-30}
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps $STEPS --warmup 5 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
exit $rc

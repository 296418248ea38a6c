#!/bin/bash
# One GPU-box pass (round 6): selected GPU tests, then bench lines.
#   TESTS="tests/test_gpu_dp.py ..." BENCH="default|none" TAG=name bash tools/gpu_pass.sh
# Every GPU step has its own time limit; the first failure ends the pass.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd "$ROOT"
O=gpurun_out/${TAG:-pass}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
      $TESTS > $O/tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" $O/tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
fi
run() {  # name, timeout, bench args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python3 bench.py "$@" > $O/bench_$n.log 2>&1 || { tail -5 $O/bench_$n.log; return 1; }
  grep '^{"metric"' $O/bench_$n.log | tail -1 > $O/bench_$n.json; cut -c1-240 $O/bench_$n.json
}
case "${BENCH:-none}" in
  default) run default 400 ;;
  *) ;;
esac

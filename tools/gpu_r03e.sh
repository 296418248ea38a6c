#!/bin/bash
# extend_nodes host overlap: unsup/pubmed GPU parity, then the Pubmed bench with phase timings.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/${TAG:-r03e}
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_unsup_ball.py tests/test_gpu_pubmed.py tests/test_apply_model.py tests/test_unsup_native.py > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
GS_UNSUP_PROF=1 timeout -k 10 300 python bench.py --config pubmed --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/prof.json" 2> "$OUT/prof.err" || exit $?
tail -4 "$OUT/prof.err"
for s in host device; do
timeout -k 10 300 python bench.py --config pubmed --steps 40 --warmup 3 --no-cpu-baseline --sampler $s > "$OUT/bench_$s.json" 2> "$OUT/bench_$s.err" || exit $?
grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_$s.json"
done

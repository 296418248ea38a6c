#!/bin/bash
# dsampler/unsup parity, Pubmed (host and device forward sampler) and its device profile.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/${TAG:-r03f}
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_dsampler.py tests/test_gpu_unsup_ball.py tests/test_gpu_pubmed.py tests/test_apply_model.py \
  tests/test_unsup_native.py tests/test_gpu_model.py > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
for s in host device; do
  timeout -k 10 300 python bench.py --config pubmed --steps 40 --warmup 3 --no-cpu-baseline --sampler $s > "$OUT/bench_$s.json" 2> "$OUT/bench_$s.err" || exit $?
  grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_$s.json"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_dev" -o run --output-format csv -- python bench.py --config pubmed --steps 20 --warmup 3 --no-cpu-baseline --sampler device > "$OUT/prof_dev.log" 2>&1 || exit $?
timeout -k 10 200 python tools/lab/ds_pubmed.py > "$OUT/ds_pubmed.txt" 2>&1 || exit $?
head -3 "$OUT/ds_pubmed.txt" | cut -c1-200

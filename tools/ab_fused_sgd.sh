#!/bin/bash
# A/B: fused slab sum + clip + SGD (GS_FUSED_SGD=1) against the two launches; parity of the fused path first.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/ab_fsgd
mkdir -p "$OUT"; cd "$ROOT"
GS_FUSED_SGD=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py > "$OUT/tests.log" 2>&1
rc=$?; tail -2 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for m in fused split; do
    if [ $m = fused ]; then export GS_FUSED_SGD=1; else unset GS_FUSED_SGD; fi
    timeout -k 10 300 python bench.py --steps 1000 --warmup 5 --no-cpu-baseline > "$OUT/b_${m}_$rep.json" 2>/dev/null || exit $?
    echo "$m rep $rep: $(grep -o '"value": [0-9.]*' "$OUT/b_${m}_$rep.json" | head -1)"
  done
done
export GS_FUSED_SGD=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --steps 300 --warmup 5 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || exit $?

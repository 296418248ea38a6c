#!/bin/bash
# Fused slab sum + clip + SGD: the whole -m gpu suite, then an A/B against
# the two-launch sequence (GS_NO_FUSED_SGD=1) and the kernel stats.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/${TAG:-r03i}
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for m in fused split; do
    if [ $m = split ]; then export GS_NO_FUSED_SGD=1; else unset GS_NO_FUSED_SGD; fi
    timeout -k 10 300 python bench.py --steps 1000 --warmup 5 --no-cpu-baseline > "$OUT/b_${m}_$rep.json" 2>/dev/null || exit $?
    echo "$m rep $rep: $(grep -o '"value": [0-9.]*' "$OUT/b_${m}_$rep.json" | head -1)"
  done
done
unset GS_NO_FUSED_SGD
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --steps 300 --warmup 5 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || exit $?

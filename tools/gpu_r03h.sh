#!/bin/bash
# bf16: wide forward tiles + W1 shadow written by the SGD.  Parity, then A/B
# of the bf16 config (chunked forward vs wide) and its kernel stats.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/${TAG:-r03h}
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_fullsize.py tests/test_gpu_model.py > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for m in chunked wide; do
    GS_LIN_FWD_BF16=$m timeout -k 10 300 python bench.py --config rmat2m-max-bf16 --steps 1000 --warmup 5 --no-cpu-baseline > "$OUT/b_${m}_$rep.json" 2>/dev/null || exit $?
    echo "$m rep $rep: $(grep -o '"value": [0-9.]*' "$OUT/b_${m}_$rep.json" | head -1)"
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --config rmat2m-max-bf16 --steps 300 --warmup 5 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || exit $?

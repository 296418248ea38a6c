#!/bin/bash
# Round-4 pass E: ublock's one-wave union stages at 8 keys per lane (the
# round-3 build that stalled a later test) on the bounded-loop build: the
# device-sampler and model GPU tests with the 8-key library, then the
# device sampler's per-batch time, 4 vs 8 keys, alternating.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r04e
mkdir -p "$OUT"; cd "$ROOT"
P=graphsage-pytorch_amd/libgraphsage_amd.so
restore() { cp tools/bin/lib_kpl4.so $P; }
trap restore EXIT
cp tools/bin/lib_kpl8.so $P
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_dsampler.py tests/test_gpu_model.py > "$OUT/tests_kpl8.log" 2>&1
rc=$?; tail -3 "$OUT/tests_kpl8.log"; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for k in 4 8; do
    cp tools/bin/lib_kpl$k.so $P
    timeout -k 10 200 python -u tools/lab/ds_time.py > "$OUT/ds_time_kpl${k}_$r.log" 2>&1 || exit $?
    echo "kpl=$k round $r: $(grep -E 'latency|back' "$OUT/ds_time_kpl${k}_$r.log" | tr '\n' ' ')"
  done
done

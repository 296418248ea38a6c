#!/bin/bash
# Device sampler state at re-entry: the rmat2m lab, hop-2 draw-workgroup
# phase stamps, rocprofv3 kernel stats of the lab.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r03ds
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 200 python -u tools/lab/ds_draw_stamps.py > "$OUT/stamps.log" 2>&1 || exit $?
cat "$OUT/stamps.log" | tail -6
TAG=r03ds bash tools/gpu_ds.sh

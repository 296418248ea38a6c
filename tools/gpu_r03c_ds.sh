#!/bin/bash
# Device sampler aux stream: parity tests + lab (GS_DS_AUX on), the lab with
# the aux stream off for comparison, rocprofv3 stats of the lab.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd "$ROOT"
OUT=$ROOT/gpurun_out/r03c_ds
mkdir -p "$OUT"
timeout -k 10 200 env GS_DS_AUX=0 python -u tools/lab/ds_time.py > "$OUT/ds_time_noaux.log" 2>&1 || exit $?
echo "no aux:"; tail -3 "$OUT/ds_time_noaux.log"
TAG=r03c_ds EXTRA_TESTS="${EXTRA_TESTS}" bash tools/gpu_ds.sh

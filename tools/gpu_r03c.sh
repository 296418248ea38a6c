#!/bin/bash
# Pubmed apply_model step with the forward's sampling on the host (helpers)
# and on the device; device sampler S=4 on rmat2m.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/${TAG:-r03c}
mkdir -p "$OUT"
cd "$ROOT"
run() {  # name, args
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err"
  local rc=$?; echo "bench $name rc=$rc"; tail -c 600 "$OUT/bench_$name.json"; echo; return $rc
}
run pub_host --config pubmed --steps 20 --warmup 3 --no-cpu-baseline || exit $?
run pub_dev --config pubmed --steps 20 --warmup 3 --no-cpu-baseline --sampler device || exit $?
run dev_s4 --gpus 1 --steps 100 --warmup 5 --no-cpu-baseline --sampler device --sampler-streams 4 --sustain 100 || exit $?

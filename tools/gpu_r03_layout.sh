#!/bin/bash
# Sampler layouts on the current step (driver's 20-step command), fp32 and
# bf16 MAX: six alternating rounds of 7:1, 12:0 and 14:0 (streams:helpers).
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
OUT=$ROOT/gpurun_out/r03layout
mkdir -p "$OUT"; cd "$ROOT"
ROUNDS=4 STEPS=20 bash tools/ab_layout_n.sh 7:1 12:0 14:0 > "$OUT/fp32.txt" 2>&1 || exit $?
tail -3 "$OUT/fp32.txt"
: > "$OUT/bf16.txt"
for i in 1 2 3; do
  for l in 7:1 12:0 14:0; do
    s=${l%%:*}; h=${l##*:}
    timeout -k 10 300 python bench.py --config rmat2m-max-bf16 --steps 300 --warmup 5 --sustain 200 --no-cpu-baseline \
        --sampler-streams $s --sampler-helpers $h > "$OUT/bf.log" 2>&1 || exit 1
    python -c "import json;d=json.loads(open('$OUT/bf.log').read().splitlines()[-1]);print('$l', d['value'], d['sustained']['value'], d['config']['sampler']['ms_per_batch'])" | tee -a "$OUT/bf16.txt"
  done
done

#!/bin/bash
# A/B of the deferred layer-2 slab sum: rocprofv3 kernel stats, both modes alternating
set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-$PWD}
for a in 1 2; do
  for m in defer split; do
    D=gpurun_out/abd_${m}_$a; mkdir -p $D
    if [ $m = split ]; then export GS_BWD_SPLIT_B=1; else unset GS_BWD_SPLIT_B; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv -- python3 bench.py --steps 300 --warmup 5 --no-cpu-baseline --sustain 300 > $D/bench.json 2>/dev/null || exit 1
    rm -f $D/run_kernel_trace.csv
  done
done

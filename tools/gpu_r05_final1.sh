#!/bin/bash
# Round-5 final pass 1: the GPU suite, then the rocprofv3 --kernel-trace
# --stats summaries of the 300-step bench command (fp32 MEAN and bf16 MAX).
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd "$ROOT"
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
for c in rmat2m rmat2m-max-bf16; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/ks_$c -o run --output-format csv -- \
      python3 bench.py --config $c --steps 300 --warmup 10 --sustain 300 --no-cpu-baseline --ref-stream-steps 0 \
      > $O/ks_$c.log 2>&1 || { tail -5 $O/ks_$c.log; exit 1; }
  tail -1 $O/ks_$c.log | cut -c1-300
done

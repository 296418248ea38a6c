#!/bin/bash
# Round-5 pass AD: the Pubmed apply_model loop with the forward's sampling on
# the device sampler against the host sampler (7 helpers), alternating.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd "$ROOT"
O=gpurun_out/r05ad
mkdir -p $O
for i in 1 2; do
  for s in host device; do
    timeout -k 10 300 python3 bench.py --config pubmed --steps 30 --warmup 3 --no-cpu-baseline --sampler $s > $O/pubmed_${s}_${i}.log 2>&1 || { tail -5 $O/pubmed_${s}_${i}.log; exit 1; }
    python3 -c "import json,sys;d=json.loads([x for x in open(sys.argv[1]).read().splitlines() if x.startswith('{')][-1]);print(sys.argv[2], d['ms_per_step'], d['config']['forward_sampler'], d['config']['extend_balls'])" $O/pubmed_${s}_${i}.log $s | tee -a $O/ab.txt
  done
done

#!/bin/bash
# Round-5 pass: GPU suite on the current build, the driver's default bench
# command twice, Pubmed twice.
set -o pipefail
O=gpurun_out/r05an
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 && tail -1 $O/gpu_tests.log &&
for i in 1 2; do timeout -k 10 300 python3 bench.py > $O/default_$i.json 2> $O/default_$i.err && tail -1 $O/default_$i.json | cut -c1-180 || exit 1; done &&
for i in 1 2; do timeout -k 10 300 python3 bench.py --config pubmed --steps 30 --warmup 3 > $O/pubmed_$i.json 2> $O/pubmed_$i.err && tail -1 $O/pubmed_$i.json | cut -c1-200 || exit 1; done

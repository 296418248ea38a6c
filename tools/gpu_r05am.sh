#!/bin/bash
# Round-5 pass: the lists job on all helpers. Sampler bench A/B (old / new
# binaries, Pubmed-sized batches with 7 helpers, rmat2m one stream + one
# helper, seven streams), GPU suite, Pubmed bench.
set -o pipefail
O=gpurun_out/r05am
mkdir -p $O
D=tools/lab/tmp_ab
for i in 1 2 3; do
  for v in old new; do
    echo "$v pubmed: $(timeout -k 10 120 $D/sb_$v 7 100 1 0 $D/pubmed.pairs 9700 10 10 | tr '\n' ' ')" >> $O/sampler_ab.txt || exit 1
  done
done
for v in old new old new; do
  echo "$v rmat2m s1h1: $(timeout -k 10 120 $D/sb_$v 1 300 1 0 | tr '\n' ' ')" >> $O/sampler_ab.txt || exit 1
  echo "$v rmat2m s7h1: $(timeout -k 10 120 $D/sb_$v 1 300 7 0 | tr '\n' ' ')" >> $O/sampler_ab.txt || exit 1
done
cat $O/sampler_ab.txt | sed 's/stream 0 phases//' | cut -c1-400
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 && tail -1 $O/gpu_tests.log &&
for i in 1 2; do timeout -k 10 300 python3 bench.py --config pubmed --steps 30 --warmup 3 --no-cpu-baseline > $O/pubmed_$i.json 2> $O/pubmed_$i.err && tail -1 $O/pubmed_$i.json | cut -c1-200 || exit 1; done

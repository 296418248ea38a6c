#!/bin/bash
# A/B of the sampler-context warm-up on the driver's bench command (20 steps).
set -o pipefail
mkdir -p gpurun_out/ab_warm
for i in 1 2 3; do
  for mode in warm cold; do
    extra=""; [ $mode = cold ] && extra="--no-warm"
    timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain 0 $extra \
      > gpurun_out/ab_warm/${mode}_$i.json 2> gpurun_out/ab_warm/${mode}_$i.err || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['config']['host_ms_per_step']['max_step'])" gpurun_out/ab_warm/${mode}_$i.json $mode
  done
done

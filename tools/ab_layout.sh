#!/bin/bash
# sampler layouts (streams:helpers) in alternating rounds: steady-window ms/step,
# value, cold-start value, sustained ms/step, sampler ms per batch, ahead at the end
mkdir -p gpurun_out
for i in 1 2; do
  for l in "$@"; do
    s=${l%%:*}; h=${l##*:}
    timeout -k 10 200 python bench.py --steps ${STEPS:-400} --warmup 10 --sustain 600 --no-cpu-baseline \
        --sampler-streams $s --sampler-helpers $h > gpurun_out/abl.log 2>&1 || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/abl.log').read().splitlines()[-1]);c=d['config'];print('$l', d['ms_per_step'], d['value'], c['cold_start']['value'], d['sustained']['ms_per_step'], c['host_ms_per_step']['sampler'], d['sustained']['sampled_ahead_at_end'])"
  done
done

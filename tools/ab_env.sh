#!/bin/bash
# A/B of runtime switches: bash tools/ab_env.sh "VAR=a" "VAR=b" ...  (3 alternating rounds)
# prints: switch, steady-window ms/step, value, sustained-window ms/step, then the event-timed
# launch means (us) of every timer site
mkdir -p gpurun_out
for i in 1 2 3; do
  for e in "$@"; do
    timeout -k 10 200 env $e python bench.py --steps 400 --warmup 10 --sustain 600 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/ab.log').read().splitlines()[-1]);print('$e', d['ms_per_step'], d['value'], d['sustained']['ms_per_step'], {k: v['avg_launch_us'] for k, v in d['roofline_kernels'].items()})"
  done
done

#!/bin/bash
# The driver's bench command N times back to back on one box (plus 300-step runs):
# the run-to-run spread of `value` that any single line sits in.
mkdir -p gpurun_out
for i in $(seq 1 ${N:-6}); do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/rep.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/rep.log').read().splitlines()[-1]);c=d['config'];print('steps20', d['value'], d['ms_per_step'], c['cold_start']['value'], d['sustained']['value'], d['roofline']['avg_launch_us'])"
done
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 300 --warmup 5 --no-cpu-baseline > gpurun_out/rep.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/rep.log').read().splitlines()[-1]);c=d['config'];print('steps300', d['value'], d['ms_per_step'], c['cold_start']['value'], d['sustained']['value'], d['roofline']['avg_launch_us'])"
done

#!/bin/bash
# A/B of the opt-in forward variants: kernel microbenchmark + in-step bench + numerics test.
mkdir -p gpurun_out
GS_LIN_FWD=wide32 timeout -k 10 200 python -m pytest -q -x -m gpu tests/test_gpu_kernels.py -k "sage_linear" -p no:cacheprovider > gpurun_out/t_wide.log 2>&1 || { tail -20 gpurun_out/t_wide.log; exit 1; }
tail -1 gpurun_out/t_wide.log
for m in none wide wide32; do
  GS_LIN_FWD=$m timeout -k 10 200 python tools/mb_linear.py --reps 50 > gpurun_out/mb_$m.txt 2>&1 || exit 1
  python -c "import json;d=json.load(open('gpurun_out/mb_$m.txt'));print('$m', d['layer1.fwd'], d['layer2.fwd'])"
done
run() {
  timeout -k 10 200 env $1 python bench.py --steps 400 --warmup 10 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab.log').read().splitlines()[-1]);print('$1', d['ms_per_step'], d['value'], d['roofline_mfma']['fwd']['avg_launch_us'])"
}
for i in 1 2; do for m in none wide32; do run "GS_LIN_FWD=$m"; done; done

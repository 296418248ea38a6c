#!/bin/bash
# A/B of runtime switches over ROUNDS alternating rounds (default 4): steady
# and sustained ms/step plus the event-timed kernels of each run, then medians.
# usage: ROUNDS=4 STEPS=300 bash tools/ab_env_k.sh "VAR=a" "VAR=b" ...
mkdir -p gpurun_out
: > gpurun_out/ab_k.txt
for i in $(seq 1 ${ROUNDS:-4}); do
  for e in "$@"; do
    timeout -k 10 200 env $e python bench.py --steps ${STEPS:-300} --warmup 10 --sustain 300 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || exit 1
    python -c "
import json;d=json.loads(open('gpurun_out/ab.log').read().splitlines()[-1]);k=d['roofline_kernels']
print('$e'.replace(' ', '+'), d['ms_per_step'], d['sustained']['ms_per_step'], k['fwd']['avg_launch_us'], k['top']['avg_launch_us'], k['dw']['avg_launch_us'], k['gather']['avg_launch_us'])" | tee -a gpurun_out/ab_k.txt
  done
done
python - <<'PY'
import collections, statistics
r = collections.defaultdict(list)
for line in open("gpurun_out/ab_k.txt"):
    f = line.split()
    r[f[0]].append([float(x) for x in f[1:]])
for k, v in r.items():
    m = [statistics.median(x[i] for x in v) for i in range(6)]
    print("median", k, "steady %.2f us  sustained %.2f us  fwd %.2f  top %.2f  dw %.2f  gather %.2f  n %d" % (m[0] * 1e3, m[1] * 1e3, m[2], m[3], m[4], m[5], len(v)))
PY

#!/bin/bash
# A/B of runtime switches over ROUNDS alternating rounds (default 6), then the
# median steady-window and sustained ms/step of each switch.
# usage: ROUNDS=6 bash tools/ab_env_n.sh "VAR=a" "VAR=b" ...
mkdir -p gpurun_out
: > gpurun_out/ab_n.txt
for i in $(seq 1 ${ROUNDS:-6}); do
  for e in "$@"; do
    timeout -k 10 200 env $e python bench.py --steps 300 --warmup 10 --sustain 300 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/ab.log').read().splitlines()[-1]);print('$e'.replace(' ', '+'), d['ms_per_step'], d['sustained']['ms_per_step'], d['roofline_kernels']['gather']['avg_launch_us'])" | tee -a gpurun_out/ab_n.txt
  done
done
python - <<'PY'
import collections, statistics
r = collections.defaultdict(list)
for line in open("gpurun_out/ab_n.txt"):
    k, a, b, g = line.split()
    r[k].append((float(a), float(b), float(g)))
for k, v in r.items():
    print("median", k, "steady", round(statistics.median(x[0] for x in v) * 1e3, 2), "us  sustained",
          round(statistics.median(x[1] for x in v) * 1e3, 2), "us  gather", round(statistics.median(x[2] for x in v), 2), "us  n", len(v))
PY

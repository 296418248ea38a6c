#!/bin/bash
# The driver's command (20 steps) under runtime switches, ROUNDS alternating
# rounds, then the median value of each switch.
mkdir -p gpurun_out
: > gpurun_out/ab20.txt
for i in $(seq 1 ${ROUNDS:-6}); do
  for e in "$@"; do
    timeout -k 10 200 env $e python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/ab.log').read().splitlines()[-1]);c=d['config'];print('$e'.replace(' ', '+'), d['value'], c['cold_start']['value'])" | tee -a gpurun_out/ab20.txt
  done
done
python - <<'PY'
import collections, statistics
r = collections.defaultdict(list)
for line in open("gpurun_out/ab20.txt"):
    k, a, b = line.split()
    r[k].append((float(a), float(b)))
for k, v in r.items():
    print("median", k, "value", round(statistics.median(x[0] for x in v) / 1e6, 3), "M  cold",
          round(statistics.median(x[1] for x in v) / 1e6, 3), "M  n", len(v))
PY

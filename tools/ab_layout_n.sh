#!/bin/bash
# Sampler layouts (streams:helpers) over ROUNDS alternating rounds at STEPS
# measured steps, then the median steady-window value of each layout.
mkdir -p gpurun_out
: > gpurun_out/abl_n.txt
for i in $(seq 1 ${ROUNDS:-6}); do
  for l in "$@"; do
    s=${l%%:*}; h=${l##*:}
    timeout -k 10 200 python bench.py --steps ${STEPS:-20} --warmup 5 --sustain 200 --no-cpu-baseline \
        --sampler-streams $s --sampler-helpers $h > gpurun_out/abl.log 2>&1 || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/abl.log').read().splitlines()[-1]);print('$l', d['value'], d['sustained']['value'])" | tee -a gpurun_out/abl_n.txt
  done
done
python - <<'PY'
import collections, statistics
r = collections.defaultdict(list)
for line in open("gpurun_out/abl_n.txt"):
    k, a, b = line.split()
    r[k].append((float(a), float(b)))
for k, v in r.items():
    print("median", k, "value", round(statistics.median(x[0] for x in v) / 1e6, 3), "M  sustained",
          round(statistics.median(x[1] for x in v) / 1e6, 3), "M  n", len(v))
PY

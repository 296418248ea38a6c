#!/bin/bash
# A/B/C... of library builds: ROUNDS alternating rounds of the bench over the
# given .so files (paths relative to the repo root), then per-build medians of
# the steady and sustained ms/step and of each timed kernel.
#   ROUNDS=3 STEPS=300 bash tools/ab_multi.sh graphsage-pytorch_amd/libgraphsage_amd.so other.so ...
mkdir -p gpurun_out
P=graphsage-pytorch_amd
cp $P/libgraphsage_amd.so /tmp/lib_main.so
: > gpurun_out/ab_multi.txt
for i in $(seq 1 ${ROUNDS:-3}); do
  for so in "$@"; do
    src=$so; [ "$so" = "$P/libgraphsage_amd.so" ] && src=/tmp/lib_main.so
    cp $src $P/libgraphsage_amd.so
    timeout -k 10 200 python bench.py --steps ${STEPS:-300} --warmup 10 --sustain ${SUSTAIN:-300} --no-cpu-baseline \
        --ref-stream-steps 0 > gpurun_out/ab.log 2>&1 || { cp /tmp/lib_main.so $P/libgraphsage_amd.so; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ab.log').read().splitlines()[-1]);print('$(basename $so)', d['ms_per_step'], d['sustained']['ms_per_step'], ' '.join(f'{k}={v[\"avg_launch_us\"]}' for k, v in d['roofline_kernels'].items()))" | tee -a gpurun_out/ab_multi.txt
  done
done
cp /tmp/lib_main.so $P/libgraphsage_amd.so
python - <<'PY'
import collections, statistics
r = collections.defaultdict(list)
for line in open("gpurun_out/ab_multi.txt"):
    f = line.split()
    r[f[0]].append([float(f[1]), float(f[2])] + [float(x.split("=")[1]) for x in f[3:]])
    names = [x.split("=")[0] for x in f[3:]]
for k, v in r.items():
    med = [statistics.median(x[i] for x in v) for i in range(len(v[0]))]
    print("median", k, "steady", round(med[0] * 1e3, 2), "us  sustained", round(med[1] * 1e3, 2), "us ",
          " ".join(f"{n} {m:.2f}" for n, m in zip(names, med[2:])), " n", len(v))
PY

#!/bin/bash
# r06 pass g: sampler layout x ring depth A/B (300 steps, the steady window is sampler-bound when
# the window's own sampling falls behind the GPU): streams / helpers / depth per stream.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/r06g
mkdir -p $O
for r in 1 2; do
  for lay in "7 1 4" "7 1 12" "10 0 12" "14 0 12" "14 0 8"; do
    set -- $lay
    tag=s$1_h$2_d$3_$r
    timeout -k 10 300 python3 bench.py --steps 300 --warmup 10 --no-cpu-baseline --ref-stream-steps 0 \
        --sampler-streams $1 --sampler-helpers $2 --sampler-depth $3 > $O/ab_$tag.log 2>&1 || { tail -5 $O/ab_$tag.log; exit 1; }
    python3 - $O/ab_$tag.log $tag <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1]
c = d["config"]; s = c["sampler"]
print(f"{sys.argv[2]}: value {d['value']/1e6:.2f} M  cold {c['cold_start']['value']/1e6:.2f}  sustained {d['sustained']['value']/1e6:.2f} M "
      f"ms/batch {s['ms_per_batch']:.3f}  capacity {s['capacity_roots_per_s']/1e6:.2f} M  wait_for_batch {c['host_ms_per_step']['wait_for_batch']*1e3:.1f} us  "
      f"step {d['ms_per_step']*1e3:.1f} us")
PY
  done
done

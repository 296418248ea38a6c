#!/bin/bash
# r06 pass c: top lab sub-stage stamps; sampler layout A/B (streams x helpers), 300 steps, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}"
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 120 tools/bin/top_lab_v4s tids > $O/top_lab_v4s.txt 2>&1; echo "lab rc=$?"; grep -A13 "stamped launch 2" $O/top_lab_v4s.txt
for v in v5 v6 v7; do
  timeout -k 10 120 tools/bin/top_lab_$v tids > $O/top_lab_$v.txt 2>&1; echo "lab $v rc=$?"; grep "per launch\|err" $O/top_lab_$v.txt | tail -3; grep -A11 "stamped launch 2" $O/top_lab_$v.txt
done
for r in 1 2; do
  for lay in "7 1" "14 0" "10 0"; do
    set -- $lay
    timeout -k 10 300 python3 bench.py --steps 300 --warmup 10 --no-cpu-baseline --ref-stream-steps 0 \
        --sampler-streams $1 --sampler-helpers $2 > $O/ab_s$1_h$2_$r.log 2>&1 || { tail -5 $O/ab_s$1_h$2_$r.log; exit 1; }
    python3 - $O/ab_s$1_h$2_$r.log $1 $2 <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1]
s = d["config"]["sampler"]
print(f"S={sys.argv[2]} h={sys.argv[3]}: value {d['value']/1e6:.2f} M  sustained {d['sustained']['value']/1e6:.2f} M "
      f"misses {d['sustained']['lookahead_misses']}  ms/batch {s['ms_per_batch']:.3f}  capacity {s['capacity_roots_per_s']/1e6:.2f} M  "
      f"step {d['ms_per_step']*1e3:.1f} us")
PY
  done
done

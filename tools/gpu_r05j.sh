#!/bin/bash
# Round-5 pass J: forward prefetch depth 2 / 3 / 4 on the balanced row split,
# judged by the in-bench per-workgroup stamps (three alternating rounds).
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd "$ROOT"
mkdir -p gpurun_out/r05j
P=graphsage-pytorch_amd
cp $P/libgraphsage_amd.so /tmp/lib_main.so
for i in 1 2 3; do
  for so in /tmp/lib_main.so $P/libgraphsage_amd_fa3.so $P/libgraphsage_amd_fa4.so; do
    cp $so $P/libgraphsage_amd.so
    timeout -k 10 300 python bench.py --steps 300 --warmup 10 --sustain 300 --no-cpu-baseline --ref-stream-steps 0 > gpurun_out/r05j/bench.log 2>&1 || { cp /tmp/lib_main.so $P/libgraphsage_amd.so; exit 1; }
    python3 -c "import json,sys;d=json.loads([x for x in open('gpurun_out/r05j/bench.log').read().splitlines() if x.startswith('{')][-1]);r=d['roofline_kernels'];print(sys.argv[1], d['ms_per_step'], d['sustained']['ms_per_step'], ' '.join(f\"{k}={v['avg_launch_us']}/{(v.get('workgroup_us') or {}).get('workgroup_mean')}\" for k,v in r.items()))" $(basename $so) | tee -a gpurun_out/r05j/ab.txt
  done
done
cp /tmp/lib_main.so $P/libgraphsage_amd.so

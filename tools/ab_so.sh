#!/bin/bash
# Build the alternative first, e.g. from graphsage-pytorch_amd/csrc: hipcc <Makefile HIPFLAGS> -D... on the
# changed kernels/*.hip, link with the other build/*.o into ../libgraphsage_amd_alt.so (see the Makefile link line).
# A/B of two builds of the library: swap the .so between bench processes.
mkdir -p gpurun_out
P=graphsage-pytorch_amd
cp $P/libgraphsage_amd.so /tmp/lib_main.so
run() {
  cp $2 $P/libgraphsage_amd.so
  timeout -k 10 300 python bench.py --steps 400 --warmup 10 --sustain 600 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab.log').read().splitlines()[-1]);print('$1', d['ms_per_step'], d['value'], d['sustained']['ms_per_step'], d['config']['final_loss'], {k: v['avg_launch_us'] for k, v in d['roofline_kernels'].items()})"
}
for i in 1 2 3; do run main /tmp/lib_main.so; run alt $P/libgraphsage_amd_alt.so; done
cp /tmp/lib_main.so $P/libgraphsage_amd.so

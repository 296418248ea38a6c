#!/bin/bash
# Build ../libgraphsage_amd_alt.so with extra -D flags on the listed kernel sources, for tools/ab_so.sh:
#   bash tools/build_alt.sh "-DGS_X=1" agg step ...
set -e
cd "$(dirname "$0")/../graphsage-pytorch_amd/csrc"
DEFS=$1; shift
H="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wall -Wno-unused-parameter -fno-gpu-rdc -munsafe-fp-atomics"
TL=/usr/local/lib/python3.10/dist-packages/torch/lib
rm -rf /tmp/alt && mkdir -p /tmp/alt
excl=""
for f in "$@"; do /opt/rocm/bin/hipcc $H $DEFS -c kernels/$f.hip -o /tmp/alt/hip_$f.o; excl="$excl|hip_$f.o"; done
objs=$(ls build/*.o | grep -v -E "${excl:1}")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../libgraphsage_amd_alt.so $objs /tmp/alt/*.o -pthread \
    -L$TL -Wl,-rpath,$TL -Wl,-rpath,/opt/rocm/lib -lamdhip64 -l:librccl.so
echo built ../libgraphsage_amd_alt.so

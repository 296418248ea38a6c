#!/bin/bash
# Build an alternative library with extra -D flags on the listed kernel sources, for tools/ab_multi.sh:
#   bash tools/build_alt.sh <out.so name under graphsage-pytorch_amd/> "-DGS_X=1" linear step ...
set -e
cd "$(dirname "$0")/../graphsage-pytorch_amd/csrc"
OUTN=$1; shift
DEFS=$1; shift
H="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wall -Wno-unused-parameter -fno-gpu-rdc -munsafe-fp-atomics"
TL=$(python3 -c "import importlib.util,os;print(os.path.join(os.path.dirname(importlib.util.find_spec('torch').origin),'lib'))")
T=$(mktemp -d /tmp/alt.XXXX)
excl=""
for f in "$@"; do /opt/rocm/bin/hipcc $H $DEFS -c kernels/$f.hip -o $T/hip_$f.o; excl="$excl|hip_$f.o"; done
objs=$(ls build/*.o | grep -v -E "${excl:1}")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../$OUTN $objs $T/*.o -pthread \
    -L$TL -Wl,-rpath,$TL -Wl,-rpath,/opt/rocm/lib -lamdhip64 -l:librccl.so
rm -rf $T
echo built ../$OUTN

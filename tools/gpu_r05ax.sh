#!/bin/bash
# Round-5 closing lines for the other configs on the final build.
set -o pipefail
O=gpurun_out/r05ax
mkdir -p $O
timeout -k 10 400 python3 bench.py --config rmat2m-max-bf16 --steps 300 --warmup 10 > $O/bf16.json 2> $O/bf16.err && tail -1 $O/bf16.json | cut -c1-160 &&
timeout -k 10 400 python3 bench.py --config rmat16m --steps 100 --warmup 10 > $O/r16.json 2> $O/r16.err && tail -1 $O/r16.json | cut -c1-160

#!/bin/bash
# Round-5 closing pass on the final build: GPU suite, smoke(), default bench.
set -o pipefail
O=gpurun_out/r05av
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 && tail -1 $O/gpu_tests.log &&
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log &&
timeout -k 10 300 python3 bench.py > $O/default.json 2> $O/default.err && tail -1 $O/default.json | cut -c1-200

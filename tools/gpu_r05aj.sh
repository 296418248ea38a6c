#!/bin/bash
# Round-5 pass: Pubmed apply_model phase breakdown (GS_UNSUP_PROF stamps) and kernel stats.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05aj
mkdir -p $O
GS_UNSUP_PROF=1 timeout -k 10 300 python3 tools/lab/pubmed_phases.py pubmed 7 > $O/phases.log 2> $O/phases.err &&
grep -v "^\[unsup\]" $O/phases.err | tail -3; tail -2 $O/phases.log && grep "\[unsup\]" $O/phases.err | tail -12 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python3 bench.py --config pubmed --steps 30 --warmup 3 --no-cpu-baseline > $O/bench.log 2>&1 && tail -1 $O/bench.log | cut -c1-300

#!/bin/bash
# Round-5 pass: the head's labels uploaded without a stream sync (Pubmed
# apply_model A/B of utils.py), then the apply_model GPU tests.
set -o pipefail
O=gpurun_out/r05aw
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -k "apply_model or unsup or model" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && tail -1 $O/tests.log &&
OUT=$O/ab BENCH_ARGS="--config pubmed --steps 30 --warmup 3" ROUNDS=3 bash tools/ab_py.sh

#!/bin/bash
# Round-5 final pass 3: the bench lines against the committed r05 profiles:
# the driver's default command, bf16 MAX 300 steps, rmat16m 100 steps, the
# Pubmed apply_model loop.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd "$ROOT"
O=gpurun_out/r05f
mkdir -p $O
run() {  # name, timeout, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python3 bench.py "$@" > $O/bench_$n.log 2>&1 || { tail -5 $O/bench_$n.log; return 1; }
  grep '^{"metric"' $O/bench_$n.log | tail -1 > $O/bench_$n.json; cut -c1-200 $O/bench_$n.json
}
run rmat2m_default 400 && run rmat2m_max_bf16_steps300 400 --config rmat2m-max-bf16 --steps 300 --no-cpu-baseline && \
run pubmed_steps30 400 --config pubmed --steps 30 --warmup 3 && \
run rmat16m_steps100 600 --config rmat16m --steps 100 --no-cpu-baseline

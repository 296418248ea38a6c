#!/bin/bash
# Round-5 final pass 2: PMC HBM traffic (FETCH_SIZE / WRITE_SIZE passes) and
# MFMA busy per kernel for fp32 MEAN and bf16 MAX, then the default bench line.
set -o pipefail
export TMPDIR=/tmp
ROOT=${GRAFT_REPO_ROOT:-$PWD}
cd "$ROOT"
O=gpurun_out/r05f
mkdir -p $O
TAG=r05_rmat2m CONFIG=rmat2m bash tools/pmc_traffic.sh > /dev/null || exit 1
TAG=r05_rmat2m bash tools/pmc_mfma.sh > /dev/null || exit 1
TAG=r05_bf16 CONFIG=rmat2m-max-bf16 BENCH_ARGS="--config rmat2m-max-bf16" bash tools/pmc_traffic.sh > /dev/null || exit 1
TAG=r05_bf16 BENCH_ARGS="--config rmat2m-max-bf16" bash tools/pmc_mfma.sh > /dev/null || exit 1
timeout -k 10 400 python3 bench.py > $O/bench_rmat2m_default.log 2>&1; rc=$?
tail -1 $O/bench_rmat2m_default.log | cut -c1-600; exit $rc

# A/B of the linear kernels in the microbenchmark under the rocprof kernel trace.
set -o pipefail
export TMPDIR=/tmp
TAG=lrand MB_ARGS="--reps 100" timeout -k 10 300 bash tools/prof_mb.sh > /dev/null && \
TAG=lcont MB_ARGS="--reps 100 --self-rows contiguous" timeout -k 10 300 bash tools/prof_mb.sh > /dev/null && \
GS_LIN_FWD=wide TAG=lwcont MB_ARGS="--reps 100 --self-rows contiguous" timeout -k 10 300 bash tools/prof_mb.sh > /dev/null

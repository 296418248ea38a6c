# A/B of the linear forward variants: parity tests, then the rocprof kernel trace of the microbenchmark.
set -o pipefail
export TMPDIR=/tmp
GS_LIN_FWD=sk timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "linear" -p no:cacheprovider > gpurun_out/t_lin_sk.log 2>&1; rc=$?; tail -1 gpurun_out/t_lin_sk.log; [ $rc -eq 0 ] || exit $rc
TAG=lrand MB_ARGS="--reps 100" timeout -k 10 300 bash tools/prof_mb.sh > /dev/null && \
GS_LIN_FWD=sk TAG=lsk MB_ARGS="--reps 100" timeout -k 10 300 bash tools/prof_mb.sh > /dev/null

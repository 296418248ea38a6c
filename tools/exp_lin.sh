# A/B of the weight-gradient slab count in the linear microbenchmark (rocprof kernel trace).
set -o pipefail
export TMPDIR=/tmp
for B in 256 512 1024; do
  GS_DW_BLOCKS=$B TAG=dw$B MB_ARGS="--reps 60" timeout -k 10 300 bash tools/prof_mb.sh > /dev/null || exit $?
done
